#!/bin/bash
# Learner + fused actor images: tests, then c5u1.  Output: gpurun_out/$1/
T=${1:-r5e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_desc_learner.py tests/test_gpu_replay_desc.py tests/test_gpu_rollout.py tests/test_gpu_rollout_graph.py $(ls tests/test_gpu_fused_actor*.py tests/test_gpu_actor*.py 2>/dev/null) -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 4 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c5u1.log 2>&1 && python tools/bench_line.py $O/bench_c5u1.log
