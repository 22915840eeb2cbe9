#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/short4; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
run w5 --steps 20 --warmup 5 --profile-every 0 && run w500 --steps 20 --warmup 500 --profile-every 0 &&
run w2000 --steps 20 --warmup 2000 --profile-every 0 && run w2000s200 --steps 200 --warmup 2000 --profile-every 0 &&
run w2000s1000 --steps 1000 --warmup 2000 --profile-every 0 && run w5s3000 --steps 3000 --warmup 5 --profile-every 0
