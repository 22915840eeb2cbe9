#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c5ch; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for c in 2 3 4 6 8; do GW_OBS_CHUNKS=$c run eager_ch$c --config c5 --steps 300 --warmup 30 --obs-eager || exit 1; done
GW_OBS_CHUNKS=4 run lazy_ch4 --config c5 --steps 300 --warmup 30 &&
GW_OBS_CHUNKS=4 GW_OBS_STREAMS=1 run eager_ch4_s1 --config c5 --steps 300 --warmup 30 --obs-eager &&
GW_OBS_CHUNKS=4 run eager_ch4_b --config c5 --steps 300 --warmup 30 --obs-eager
