#!/bin/bash
# the driver's command (C3, 20 steps, warmup 5) under a kernel trace without the profiled steps after the timed region: where a short run's time goes (tools/run_span.py)
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r6span; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --profile-steps 0 --no-cpu-baseline > $O/bench$i.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/run_span.py $(find $O/t$i -name "run_kernel_trace.csv" | head -1) 20 > $O/span$i.txt
python3 $GRAFT_REPO_ROOT/tools/timeline.py $(find $O/t$i -name "run_kernel_trace.csv" | head -1) step_v2 25 > $O/timeline$i.txt
done
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --profile-steps 0 --no-cpu-baseline > $O/bench_noprof.log 2>&1
