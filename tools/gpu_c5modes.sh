#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c5modes; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
run lazy --config c5 --steps 300 --warmup 30 && run eager --config c5 --steps 300 --warmup 30 --obs-eager &&
GW_OBS_CHUNKS=4 run eager_ch4 --config c5 --steps 300 --warmup 30 --obs-eager &&
GW_OBS_CHUNKS=2 run lazy_ch2 --config c5 --steps 300 --warmup 30 && GW_OBS_STREAMS=1 run lazy_s1 --config c5 --steps 300 --warmup 30 &&
run bf16 --config c5 --steps 300 --warmup 30 --obs-dtype bf16
