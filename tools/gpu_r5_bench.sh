#!/bin/bash
# Round-5 bench lines: c5u1, c4patch, c5patch, c3 (no CPU baseline).  Output: gpurun_out/$1/
T=${1:-r5bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for c in "c5 --updates-per-step 1 --steps 100 --warmup 20" "c4patch --steps 200 --warmup 20" "c5patch --steps 200 --warmup 20" "c3 --steps 20 --warmup 5"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$n.log 2>&1 || exit 1
  python tools/bench_line.py $O/bench_$n.log
done
