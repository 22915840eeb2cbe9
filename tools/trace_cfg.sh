#!/bin/bash
# rocprofv3 kernel trace of one bench config (no PMC) + the per-step timeline.  Usage: tools/trace_cfg.sh TAG [bench args]
TAG=${1:-t}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $ROOT/bench.py "$@" --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
python3 $ROOT/tools/timeline.py $(find $OUT -name "run_kernel_trace.csv" | head -1) ${ANCHOR:-act_kernel} 4 > $OUT/timeline.txt
tail -1 $OUT/bench.log | cut -c1-300
