#!/bin/bash
# The step's windows from the FeAR launch (gw_step_patch_next): tests, then c5patch with it
# (default) vs the writer after the step (GW_FEAR_PATCH=0).
T=${1:-r5fp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_obs_patch.py tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $s; }
for fp in 1 0 1 0; do
  GW_FEAR_PATCH=$fp timeout -k 10 300 python bench.py --config c5patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c5p_$fp.log 2>&1 || exit 1
  echo "fear_patch=$fp $(python tools/bench_line.py $O/c5p_$fp.log | tr '\n' ' ' | tr -s ' ' | cut -c1-400)"
done
