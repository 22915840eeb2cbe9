#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/d20; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for rep in 1 2 3; do run d20_$rep --steps 20 --warmup 5 && run d20p0_$rep --steps 20 --warmup 5 --profile-every 0 || exit 1; done
run s1000 --steps 1000 --warmup 100
