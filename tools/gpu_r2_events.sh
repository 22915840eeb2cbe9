#!/bin/bash
# Round 2: pipeline events without the system-scope fence, launch-carried profiling events,
# HIP return compaction.  Bench lines (driver size and long), C2 sync / async / graph, and a
# rocprofv3 kernel trace + stats of the default command.  gpurun_out/r2_events/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r2_events; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
for rep in 1 2 3; do run d20_$rep --steps 20 --warmup 5 || exit 1; done
run s1000 --steps 1000 --warmup 100 &&
run c2 --config c2 &&
run c2_async --config c2 --obs-eager --graph 0 &&
run c2_lazy --config c2 --obs-lazy --graph 0 &&
run c2_eager_sync --config c2 --graph 0 &&
run c1 --config c1 &&
run c1_eager --config c1 --graph 0 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --no-cpu-baseline > $O/prof.log 2>&1 && tail -n 1 $O/prof.log | cut -c1-200 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python bench.py --config c2 --graph 0 --obs-eager --no-cpu-baseline > $O/prof_c2.log 2>&1 && ls $O/prof
