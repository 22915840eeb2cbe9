#!/bin/bash
# c5u1: the obs writer's first launch as a share of its blocks (GW_OBS_FIRST, %) with 2 / 3 launches.
T=${1:-r5first}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for v in "2 0" "2 25" "2 35" "3 30" "2 0" "2 25" "2 35" "3 30"; do
  set -- $v
  GW_OBS_CHUNKS=$1 GW_OBS_FIRST=$2 timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c$1_$2.log 2>&1 || exit 1
  echo "chunks $1 first $2: $(python tools/bench_line.py $O/c$1_$2.log | head -1)"
done
