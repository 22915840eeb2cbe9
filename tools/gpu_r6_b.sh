#!/bin/bash
# Round 6: obs-writer parity subset + C3 bench lines (table-based writer, value-select fix).
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async_obs.py tests/test_gpu_bench_mode.py tests/test_gpu_obs_bf16.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_20.log 2>&1 || { tail -5 $O/c3_20.log; exit 1; }
timeout -k 10 120 python bench.py --steps 1000 --warmup 50 --no-cpu-baseline > $O/c3_1000.log 2>&1 || { tail -5 $O/c3_1000.log; exit 1; }
timeout -k 10 200 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
