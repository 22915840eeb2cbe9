#!/bin/bash
# FeAR sims with per-lane pair lists (N > 4): parity tests, then c4patch / c4 with FeAR on, same-box A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/flist; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async_obs.py tests/test_gpu_obs_bf16.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
LIBS="head=marl-responsible-nav_amd/csrc/build_ab/head/libgridenv.so cur=" bash tools/gpu_ab.sh flist/c4pf c4patch --fear 1 --steps 100 --warmup 10 || exit 1
LIBS="head=marl-responsible-nav_amd/csrc/build_ab/head/libgridenv.so cur=" bash tools/gpu_ab.sh flist/c4f c4 --fear 1 --steps 100 --warmup 10
