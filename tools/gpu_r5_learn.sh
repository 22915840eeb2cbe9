#!/bin/bash
# Descriptor learner timing without stamps (3 repeats) and the c5u1 bench line.
T=${1:-r5learn}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_desc_learn.py 65536 200 > $O/learn$i.log 2>&1 || { tail -5 $O/learn$i.log; exit 1; }
  tail -1 $O/learn$i.log
done
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 20 --no-cpu-baseline > $O/c5u1.log 2>&1 || exit 1
python tools/bench_line.py $O/c5u1.log
