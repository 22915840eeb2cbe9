#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/wide; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for rep in 1 2 3; do
run f32_$rep && GW_FEAR_BE=wide run f32w_$rep || exit 1
done
run d20 --steps 20 --warmup 5 && GW_FEAR_BE=wide run d20w --steps 20 --warmup 5 &&
run c5 --config c5 --steps 300 --warmup 30 && GW_FEAR_BE=wide run c5w --config c5 --steps 300 --warmup 30 &&
run c4f --config c4f --steps 300 --warmup 30 && GW_FEAR_BE=wide run c4fw --config c4f --steps 300 --warmup 30
