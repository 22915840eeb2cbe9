#!/bin/bash
# c5: the fused actor's grid capped at fewer blocks (GW_ACT_RESIDENT), leaving CUs to the obs writer.
T=${1:-r5actres}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for r in 256 192 128 96 256 192 128 96; do
  GW_ACT_RESIDENT=$r timeout -k 10 300 python bench.py --config c5 --steps 100 --warmup 20 --no-cpu-baseline > $O/c5_$r.log 2>&1 || exit 1
  echo "resident $r: $(python tools/bench_line.py $O/c5_$r.log | tr '\n' ' ' | tr -s ' ' | cut -c1-330)"
done
