#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/misc; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_obs_bf16.py tests/test_gpu_async_obs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
run bf16 --obs-dtype bf16 && run bf16b --obs-dtype bf16 &&
timeout -k 10 120 python tools/bench_learn.py 128 > $O/learn.log 2>&1; tail -3 $O/learn.log
run c5u1 --config c5 --steps 100 --warmup 10 --updates-per-step 1
