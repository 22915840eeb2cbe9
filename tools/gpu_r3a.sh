#!/bin/bash
# Round-3 changes: learner / DP / dist / rollout tests, driver bench line, the 2-rank gloo bench
# rehearsal (launched by bench.py itself) and its rocprofv3 kernel stats.  gpurun_out/r3a/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_maddpg.py tests/test_maddpg_dp.py tests/test_gpu_dist.py tests/test_gpu_rollout.py tests/test_gpu_ln_relu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 && python tools/bench_line.py $O/bench_driver.log driver &&
MARLNAV_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gloo2.log 2>&1 && tail -c 400 $O/bench_gloo2.log &&
MARLNAV_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c5 --steps 20 --warmup 5 --updates-per-step 1 > $O/bench_gloo2_c5.log 2>&1 && tail -c 400 $O/bench_gloo2_c5.log &&
cd /tmp && export TMPDIR=/tmp && MARLNAV_DIST_BACKEND=gloo timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gloo2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 2 --config c5 --steps 20 --warmup 5 > $O/prof_gloo2.log 2>&1; echo "rocprof rc $?"
