#!/bin/bash
# Measurement only: libgridenv with gridenv.hip taken from git revision REV (default HEAD), the other
# objects from the current build -> csrc/build_ab/REV/libgridenv.so.  Load it with MARLNAV_LIB=<path>
# for a same-box A/B against the working tree's library (tools/gpu_ab.sh).
set -e
REV=${1:-HEAD}   # a git revision, or wt = the working tree's gridenv.hip
XF=${2:-}       # extra compile flags (e.g. -DGW_NOFEAR_BE=16); the output dir is REV$TAG
TAG=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/marl-responsible-nav_amd/csrc
O=$C/build_ab/$REV$TAG
mkdir -p $O
if [ "$REV" = wt ]; then cp $C/gridenv.hip $O/gridenv.hip
else git -C $R show $REV:marl-responsible-nav_amd/csrc/gridenv.hip > $O/gridenv.hip; fi
cp $C/*.h $O/
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -I$R/include"
/opt/rocm/bin/hipcc $F $XF -c $O/gridenv.hip -o $O/gridenv.o
objs=""
for s in learner_ops actor_ops rollout_ops maddpg_ops patch_ops; do
  o=$(ls -t $C/build/$s.*.o | head -1); objs="$objs $o"
done
/opt/rocm/bin/hipcc $F -shared $O/gridenv.o $objs -o $O/libgridenv.so
echo built $O/libgridenv.so
