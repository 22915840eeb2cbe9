#!/bin/bash
# The CNN head's listing beside the window writer: tests, then c4patch with the side listing
# (default) vs the act listing itself (GW_CNN_LIST_SIDE=0).
T=${1:-r5list}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch_cnn.py tests/test_gpu_obs_patch.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $s; }
for side in 1 0 1 0; do
  GW_CNN_LIST_SIDE=$side timeout -k 10 300 python bench.py --config c4patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c4p_$side.log 2>&1 || exit 1
  echo "side=$side $(python tools/bench_line.py $O/c4p_$side.log | head -1)"
done
