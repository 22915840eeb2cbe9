#!/bin/bash
# Round 6: GPU suite + C3 bench (table-based obs writer) + C5 actor block-size A/B (GW_ACT_WAVES).
set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_20.log 2>&1 || { tail -5 $O/c3_20.log; exit 1; }
timeout -k 10 120 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline > $O/c3_1000.log 2>&1 || { tail -5 $O/c3_1000.log; exit 1; }
for w in 16 12 8; do
  GW_ACT_WAVES=$w timeout -k 10 200 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/c5_w$w.log 2>&1 || { tail -5 $O/c5_w$w.log; exit 1; }
done
