#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/nowar; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for rep in 1 2; do run c3_$rep && GW_MEASURE_NO_WAR=1 run c3nw_$rep || exit 1; done
run bf16 --obs-dtype bf16 && GW_MEASURE_NO_WAR=1 run bf16nw --obs-dtype bf16
