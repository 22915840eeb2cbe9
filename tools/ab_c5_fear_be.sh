#!/bin/bash
O=gpurun_out/ab_c5fear; mkdir -p $O
for i in 1 2; do for b in wide narrow; do
  GW_FEAR_BE=$b timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/c5_${b}_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c5_${b}_$i.log | sed "s/^/$b /" | tee -a $O/summary.txt
done; done
