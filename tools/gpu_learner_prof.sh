#!/bin/bash
# rocprofv3 kernel trace + stats of tools/bench_next.py f1 (the learner update) -> gpurun_out/learner/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/learner; mkdir -p $O; R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/tools/bench_next.py f1 > $O/prof.log 2>&1 &&
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/f1_kernel_stats.csv \; && tail -n 1 $O/prof.log
