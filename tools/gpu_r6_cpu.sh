#!/bin/bash
# Round 6: each config's bench line WITH its CPU baseline (the C restatement on the host cores), for BASELINE.md section 4.  Output: gpurun_out/$1/
T=${1:-r6cpu}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for c in "c1 --steps 500 --warmup 50" "c2 --steps 500 --warmup 50" "c4 --steps 20 --warmup 5" "c4f --steps 20 --warmup 5" "c5 --steps 100 --warmup 20" "c4patch --steps 200 --warmup 20"; do
  n=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 8 > $O/$n.log 2>&1 || exit 1
  python tools/summ.py $O/$n.log | tee -a $O/summary.txt
done
