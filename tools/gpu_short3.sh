#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/short3; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
run s20p0 --steps 20 --warmup 5 --profile-every 0 && run s200p0 --steps 200 --warmup 5 --profile-every 0 &&
run s1000p0 --steps 1000 --warmup 5 --profile-every 0 && run s1000 --steps 1000 --warmup 100 &&
run s20 --steps 20 --warmup 5 && run s20ng --steps 20 --warmup 5 --no-gather --profile-every 0
