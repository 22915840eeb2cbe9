#!/bin/bash
# The window writer and the CNN head's listing in one launch: tests, then c4patch with it (default)
# vs the separate writer and act (GW_CNN_WRITE_LIST=0).
T=${1:-r5wl}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch_cnn.py tests/test_gpu_obs_patch.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $s; }
for wl in 1 0 1 0; do
  GW_CNN_WRITE_LIST=$wl timeout -k 10 300 python bench.py --config c4patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c4p_$wl.log 2>&1 || exit 1
  echo "write_list=$wl $(python tools/bench_line.py $O/c4p_$wl.log | tr '\n' ' ' | tr -s ' ' | cut -c1-400)"
done
