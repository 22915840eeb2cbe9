#!/bin/bash
# Round 6: C5 with 128-VGPR 12 / 8-wave actor blocks (act_kernel_lean), FeAR joined / async; c4patch check.
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_actor_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for cfg in "16 -" "12 -" "8 -" "8 --fear-async" "12 --fear-async" "16 -" "8 -"; do
  set -- $cfg; fa=$2; [ "$fa" = "-" ] && fa=""
  tag=c5_w$1$fa
  GW_ACT_WAVES=$1 timeout -k 10 200 python bench.py --config c5 $fa --steps 200 --warmup 20 --no-cpu-baseline > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python /root/repo/tools/summ.py $O/$tag.log >> $O/summary.txt
done
timeout -k 10 200 python bench.py --config c4patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c4patch.log 2>&1 || { tail -5 $O/c4patch.log; exit 1; }
python /root/repo/tools/summ.py $O/c4patch.log >> $O/summary.txt
