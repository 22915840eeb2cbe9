#!/bin/bash
# Round 6: the C2 actor launch carrying the queued obs writer -- its tests, then a same-box A/B (GW_ACT_OBS=0 / 1)
O=gpurun_out/r6c2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rollout_graph.py tests/test_gpu_bench_c5_c2.py tests/test_actor_ops.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do for a in 0 1; do
  GW_ACT_OBS=$a timeout -k 10 300 python bench.py --config c2 --steps 500 --warmup 50 --no-cpu-baseline > $O/c2_ao${a}_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c2_ao${a}_$i.log | sed "s/^/ao$a /" | tee -a $O/summary.txt
done; done
