#!/bin/bash
# step_v2 phase stamps (measurement build, tools/step_clk.sh): C2's shape and c4patch's (N = 8, no dense obs)
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/marl-responsible-nav_amd/csrc/build_clk/libgridenv_clk.so
MARLNAV_LIB=$L timeout -k 10 120 python tools/step_clk.py 4096 40 merged grid32 32 || exit 1
MARLNAV_LIB=$L timeout -k 10 120 python tools/step_clk.py 65536 40 noobs grid64_n8 128 || exit 1
MARLNAV_LIB=$L timeout -k 10 120 python tools/step_clk.py 65536 40 noobs grid32 32
