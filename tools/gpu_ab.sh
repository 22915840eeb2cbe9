#!/bin/bash
# Same-box A/B of libgridenv builds (tools/ab_lib.sh): LIBS="name=path name=path ..." (path relative
# to the repo; an empty path = the working tree's library).  Rounds of alternating bench runs of one
# config, then (c2) rocprofv3 kernel stats of tools/c2_probe.py per library.
# Usage: LIBS="a=marl-responsible-nav_amd/csrc/build_ab/HEAD/libgridenv.so b=" tools/gpu_ab.sh TAG CONFIG [bench args...]
T=$1; CFG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T; mkdir -p $O
run() {  # name path cmd...
  local n=$1 p=$2; shift 2
  if [ -n "$p" ]; then MARLNAV_LIB=$ROOT/$p "$@"; else "$@"; fi
}
for i in 1 2 3; do
  for nv in $LIBS; do
    n=${nv%%=*}; p=${nv#*=}
    run $n "$p" timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline "$@" > $O/${n}_$i.log 2>&1 && python tools/bench_line.py $O/${n}_$i.log ${n}_$i || exit 1
  done
done
[ "$CFG" = c2 ] || exit 0
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  for nv in $LIBS; do
    n=${nv%%=*}; p=${nv#*=}
    run $n "$p" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${n}_prof$m -o run --output-format csv -- python3 $ROOT/tools/c2_probe.py $m > $O/${n}_prof$m.log 2>&1 || exit 1
    f=$(find $O/${n}_prof$m -name '*kernel_stats.csv' | head -n 1); echo "$n mode $m: $(sed -n 2p "$f" | cut -d, -f1,4,6,7)"
  done
done
