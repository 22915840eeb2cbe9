#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/cross2; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
for e in 8192 16384 24576 32768; do
  GW_KERNEL=merged run m_$e --envs $e --steps 500 --warmup 50 &&
  GW_KERNEL=defer run d_$e --envs $e --steps 500 --warmup 50 --obs-eager || exit 1
done
run c5_s2 --config c5 --steps 300 --warmup 30 && GW_OBS_STREAMS=1 run c5_s1 --config c5 --steps 300 --warmup 30 &&
run c5_eager --config c5 --steps 300 --warmup 30 --obs-eager && run c4cnn --config c4cnn --steps 200 --warmup 20 &&
GW_OBS_STREAMS=1 run c4cnn_s1 --config c4cnn --steps 200 --warmup 20 && run c5patch --config c5patch --steps 300 --warmup 30
