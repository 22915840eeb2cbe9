#!/bin/bash
# Learner iteration: the learner's tests, then its rocprofv3 profile (tools/gpu_r5_lprof.sh).
T=${1:-r5s}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_desc_learner.py tests/test_maddpg_fused.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 4 $O/pytest.log; [ $s = 0 ] || exit $s
bash $GRAFT_REPO_ROOT/tools/gpu_r5_lprof.sh $T
