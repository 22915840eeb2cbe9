#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats, then one PMC pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), and a VALU pass (3 SQ + 1 GRBM counters).  Usage: tools/gpu_profile.sh TAG [bench args]
TAG=${1:-r1}; shift
ARGS=${@:---steps 50 --warmup 10}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
echo "== trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $OUT/trace.log 2>&1 && tail -1 $OUT/trace.log &&
echo "== fetch" && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $OUT/fetch.log 2>&1 &&
echo "== write" && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $OUT/write.log 2>&1 &&
echo "== valu" && timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- python3 $ROOT/bench.py $ARGS --no-cpu-baseline > $OUT/valu.log 2>&1 &&
echo "== done" && find $OUT -name "*.csv" | head -20
