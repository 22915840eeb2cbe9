#!/bin/bash
# Measurement build (never loaded by the product path): libgridenv with GW_STEP_CLK phase stamps in
# step_v2_block -> csrc/build_clk/libgridenv_clk.so; load it with MARLNAV_LIB=<path> (tools/step_clk.py).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/marl-responsible-nav_amd/csrc
O=$C/build_clk
mkdir -p $O
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -I$R/include"
/opt/rocm/bin/hipcc $F -DGW_STEP_CLK -c $C/gridenv.hip -o $O/gridenv_clk.o
objs=""
for s in learner_ops actor_ops rollout_ops maddpg_ops patch_ops; do
  o=$(ls -t $C/build/$s.*.o | head -1); objs="$objs $o"
done
/opt/rocm/bin/hipcc $F -shared $O/gridenv_clk.o $objs -o $O/libgridenv_clk.so
echo built $O/libgridenv_clk.so
