#!/bin/bash
# near-pair list resolve (N > 4): parity tests, then c4patch / c4 same-box A/B against build_ab/HEAD
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/list; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async_obs.py tests/test_gpu_patch_cnn.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
LIBS="head=marl-responsible-nav_amd/csrc/build_ab/HEAD/libgridenv.so cur=" bash tools/gpu_ab.sh list/c4p c4patch --steps 100 --warmup 10 || exit 1
LIBS="head=marl-responsible-nav_amd/csrc/build_ab/HEAD/libgridenv.so cur=" bash tools/gpu_ab.sh list/c4 c4 --steps 100 --warmup 10
