#!/bin/bash
# rocprofv3 kernel trace of the descriptor learner alone.  Output: gpurun_out/$1/
T=${1:-r5lp}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python $GRAFT_REPO_ROOT/tools/bench_desc_learn.py 65536 100 > $O/learn.log 2>&1 && cat $O/learn.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_desc_learn.py 65536 100 > $O/prof.log 2>&1 &&
f=$(find $O/prof -name '*kernel_stats.csv' | head -1) && cp $f $O/learn_kernel_stats.csv && head -12 $O/learn_kernel_stats.csv | cut -c1-200
