#!/bin/bash
# Round 6: narrow FeAR blocks for envs without a full-obs writer (gw_set_fear_blocks) -- the GPU suite, then c5patch / c4patch lines
O=gpurun_out/r6fb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c5patch_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c5patch_$i.log | tee -a $O/summary.txt
done
timeout -k 10 300 python bench.py --config c4patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c4patch.log 2>&1 || exit 1
python tools/summ.py $O/c4patch.log | tee -a $O/summary.txt
