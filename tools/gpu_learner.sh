#!/bin/bash
# Learner (§8f row 1): the HIP LayerNorm+ReLU epilogue and the frozen-critic actor loss.
# Parity tests, then the batch-128 update timed with the epilogue on and off, then a rocprofv3
# kernel trace of the graph-replayed update.  gpurun_out/learner/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/learner; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ln_relu.py tests/test_maddpg.py tests/test_gpu_replay.py tests/test_gpu_rollout.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
GW_LN_FUSED=1 timeout -k 10 120 python tools/bench_next.py f1 > $O/f1_fused.log 2>&1 && cat $O/f1_fused.log &&
timeout -k 10 120 python tools/bench_next.py f1 > $O/f1_torchln.log 2>&1 && cat $O/f1_torchln.log &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_next.py f1 > $O/prof.log 2>&1 &&
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/f1_kernel_stats.csv \; && head -25 $O/f1_kernel_stats.csv
