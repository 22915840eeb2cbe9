#!/bin/bash
# Pipeline events bound to the kernel launches (GW_BIND_EVENTS=1, default) vs marker records:
# the async-obs parity tests, then bench A/B and a kernel trace.  gpurun_out/bind/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/bind; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_bench_mode.py tests/test_gpu_obs_bf16.py tests/test_gpu_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
for rep in 1 2; do
run c3_$rep --steps 1000 --warmup 100 &&
GW_BIND_EVENTS=0 run c3_nobind_$rep --steps 1000 --warmup 100 || exit 1
done
run d20 --steps 20 --warmup 5 &&
run bf16 --obs-dtype bf16 &&
run c5 --config c5 --steps 300 --warmup 30 &&
run c4 --config c4 --steps 300 --warmup 30 &&
run c4cnn --config c4cnn --steps 200 --warmup 20 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --no-cpu-baseline --profile-every 0 > $O/prof.log 2>&1 && python tools/gaps.py $O/prof/c3_kernel_trace.csv
