#!/bin/bash
# Quick bench lines: C3 (long and driver size), C2, C5, bf16.  gpurun_out/quick/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/quick; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
run c3 --steps 1000 --warmup 100 && run d20 --steps 20 --warmup 5 && run c2 --config c2 && run c2b --config c2 &&
GW_BIND_EVENTS=0 run c3_nobind --steps 1000 --warmup 100 &&
run c5 --config c5 --steps 300 --warmup 30 && run bf16 --obs-dtype bf16 && run c1 --config c1
