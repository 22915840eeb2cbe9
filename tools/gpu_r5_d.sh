#!/bin/bash
# Descriptor learner tests + block stamps + learner kernel profile.  Output: gpurun_out/$1/
T=${1:-r5d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_desc_learner.py -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 4 $O/pytest.log; [ $s = 0 ] || exit $s
bash $R/tools/gpu_r5_stamp.sh $T || exit 1
bash $R/tools/gpu_r5_lprof.sh $T
