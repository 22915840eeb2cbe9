#!/bin/bash
# c5u1: the obs writer as 1 / 2 (default) / 4 / 8 launches per step (GW_OBS_CHUNKS).
T=${1:-r5chunks}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for c in 2 4 8 1 2 4 8; do
  GW_OBS_CHUNKS=$c timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c$c.log 2>&1 || exit 1
  echo "chunks $c: $(python tools/bench_line.py $O/c$c.log | head -1)"
done
