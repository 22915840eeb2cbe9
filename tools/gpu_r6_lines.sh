#!/bin/bash
# Round-6 bench lines for every config (no CPU baseline) + the C3 line with it.  Output: gpurun_out/$1/
T=${1:-r6lines}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for c in "c3 --steps 20 --warmup 5" "c3 --steps 1000 --warmup 20" "c5 --steps 100 --warmup 20" "c5 --updates-per-step 1 --steps 100 --warmup 20" "c4patch --steps 200 --warmup 20" "c5patch --steps 200 --warmup 20" "c2 --steps 500 --warmup 50" "c4f --steps 20 --warmup 5" "c4 --steps 20 --warmup 5" "c1 --steps 500 --warmup 50" "c4cnn --steps 20 --warmup 5"; do
  n=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/$n.log 2>&1 || exit 1
  python tools/summ.py $O/$n.log | tee -a $O/summary.txt
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/c3_cpu.log 2>&1 || exit 1
