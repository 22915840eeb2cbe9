#!/bin/bash
# Round 6: writer tables for the step obs only (terminal obs by the compare loop): parity, then C3 / C5 / C5+update lines.
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async_obs.py tests/test_gpu_bench_mode.py tests/test_gpu_obs_bf16.py tests/test_gpu_replay.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for c in "c3 --steps 1000 --warmup 20" "c3 --steps 20 --warmup 5" "c5 --steps 200 --warmup 20" "c5 --updates-per-step 1 --steps 100 --warmup 20" "c3 --steps 20 --warmup 5"; do
  n=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  python tools/summ.py $O/$n.log >> $O/summary.txt
done
