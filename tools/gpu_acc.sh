#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/acc; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_dist.py tests/test_gpu_replay.py tests/test_gpu_async_obs.py tests/test_maddpg.py tests/test_gpu_obs_patch.py tests/test_gpu_cnn_actor.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
run c5_1 --config c5 --steps 300 --warmup 30 && run c5_2 --config c5 --steps 300 --warmup 30 && run c4cnn --config c4cnn --steps 200 --warmup 20
