#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/split2; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
run bf16_defer --obs-dtype bf16 && GW_KERNEL=split run bf16_split --obs-dtype bf16 --obs-eager &&
GW_KERNEL=defer GW_FEAR_BE=wide run bf16_wide --obs-dtype bf16 &&
run f32_defer && GW_KERNEL=split run f32_split --obs-eager && GW_KERNEL=defer GW_FEAR_BE=wide run f32_wide &&
GW_KERNEL=split run bf16_split_ring2 --obs-dtype bf16 --obs-eager --obs-ring 2 && run bf16_ring1 --obs-dtype bf16 --obs-ring 1
