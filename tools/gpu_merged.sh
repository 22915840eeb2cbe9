#!/bin/bash
# GW_KERNEL=merged (one step_obs launch per step) vs the default defer pipeline: parity tests
# first, then bench A/B.  gpurun_out/merged/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/merged; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_obs_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k merged > $O/pytest_parity.log 2>&1; s=$?; tail -n 2 $O/pytest_parity.log; [ $s = 0 ] || exit $s
run c3 --steps 1000 --warmup 100 &&
GW_KERNEL=merged run c3_m --steps 1000 --warmup 100 &&
GW_KERNEL=merged GW_MERGE_ORDER=1 run c3_m1 --steps 1000 --warmup 100 &&
GW_KERNEL=merged GW_OBS_BE=2 run c3_mbe2 --steps 1000 --warmup 100 &&
GW_KERNEL=merged GW_OBS_BE=8 run c3_mbe8 --steps 1000 --warmup 100 &&
GW_KERNEL=merged run d20_m --steps 20 --warmup 5 &&
run d20 --steps 20 --warmup 5 &&
GW_KERNEL=merged run c2_m --config c2 &&
GW_KERNEL=merged run bf16_m --obs-dtype bf16 &&
run bf16 --obs-dtype bf16 &&
GW_KERNEL=merged run c5_m --config c5 --steps 300 --warmup 30 &&
GW_KERNEL=merged run c4_m --config c4 --steps 300 --warmup 30 &&
run c4 --config c4 --steps 300 --warmup 30 &&
GW_KERNEL=merged run c4f_m --config c4f --steps 300 --warmup 30 &&
run c4f --config c4f --steps 300 --warmup 30 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
GW_KERNEL=merged timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3m -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 > $O/prof.log 2>&1 && ls $O/prof
