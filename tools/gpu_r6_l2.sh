#!/bin/bash
# Round 6: L2 hit / miss of the C5 kernels (is the actor's W1 gather evicted by the obs writer?).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r6_l2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/c5 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 30 --warmup 10 --no-cpu-baseline > $OUT/c5.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/c3 -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 30 --warmup 10 --no-cpu-baseline > $OUT/c3.log 2>&1 || exit 1
