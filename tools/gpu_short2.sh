#!/bin/bash
# Where a short timed region loses time: warmup length and step count sweep.  gpurun_out/short2/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/short2; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for rep in 1 2; do
run s20w5_$rep --steps 20 --warmup 5 && run s20w100_$rep --steps 20 --warmup 100 &&
run s20w5p0_$rep --steps 20 --warmup 5 --profile-every 0 && run s40w5_$rep --steps 40 --warmup 5 &&
run s80w5_$rep --steps 80 --warmup 5 && run s20w5ng_$rep --steps 20 --warmup 5 --no-gather || exit 1
done
