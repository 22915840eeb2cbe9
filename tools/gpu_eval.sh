#!/bin/bash
# Evaluation driver (§8f row 2): parity test and throughput.  gpurun_out/eval/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/eval; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/bench_next.py f2 > $O/f2.log 2>&1 && grep row $O/f2.log
