#!/bin/bash
# Round 6: the async obs writer on a CU subset (GW_OBS_CUS) at C5 and C3.
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
for n in 0 64 96 128 192; do
  GW_OBS_CUS=$n timeout -k 10 200 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/c5_cu$n.log 2>&1 || { tail -5 $O/c5_cu$n.log; exit 1; }
  python /root/repo/tools/summ.py $O/c5_cu$n.log >> $O/summary.txt
done
for n in 0 128 192; do
  GW_OBS_CUS=$n timeout -k 10 200 python bench.py --config c3 --steps 500 --warmup 20 --no-cpu-baseline > $O/c3_cu$n.log 2>&1 || { tail -5 $O/c3_cu$n.log; exit 1; }
  python /root/repo/tools/summ.py $O/c3_cu$n.log >> $O/summary.txt
done
