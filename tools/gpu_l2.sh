#!/bin/bash
# world update per-lane pair lists for N <= 4 too (-DGW_LIST_MIN_N=2): C2 and C3 same-box A/B + the C2 parity tests
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/l2; mkdir -p $O
MARLNAV_LIB=$R/marl-responsible-nav_amd/csrc/build_ab/wt_l2/libgridenv.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_c5_c2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
LIBS="l2=marl-responsible-nav_amd/csrc/build_ab/wt_l2/libgridenv.so cur=" bash tools/gpu_ab.sh l2/c2 c2 --steps 200 --warmup 20 || exit 1
LIBS="l2=marl-responsible-nav_amd/csrc/build_ab/wt_l2/libgridenv.so cur=" bash tools/gpu_ab.sh l2/c3 c3 --steps 100 --warmup 10
