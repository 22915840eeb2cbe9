#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c5ab2; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for rep in 1 2; do
run c5_$rep --config c5 --steps 300 --warmup 30 && run c5fa_$rep --config c5 --steps 300 --warmup 30 --fear-async &&
GW_OBS_STREAMS=1 run c5fa_s1_$rep --config c5 --steps 300 --warmup 30 --fear-async || exit 1
done
