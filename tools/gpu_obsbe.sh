#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/obsbe; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for rep in 1 2; do
run be4_$rep && GW_OBS_BE=2 run be2_$rep && GW_OBS_BE=8 run be8_$rep && GW_OBS_NT=0 run plain_$rep &&
run ring3_$rep --obs-ring 3 || exit 1
done
