#!/bin/bash
# fused learner: tests, timing fused vs autograd, rocprofv3 stats of graph-replayed updates. gpurun_out/r3d/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_maddpg_fused.py tests/test_maddpg.py tests/test_maddpg_dp.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; grep -E "rel L2|worst|passed|failed|Error" $O/pytest.log | head -20; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/bench_learn.py 128 fused > $O/learn.log 2>&1 && timeout -k 10 120 python tools/bench_learn.py 128 autograd >> $O/learn.log 2>&1 && cat $O/learn.log &&
timeout -k 10 300 python bench.py --config c5 --steps 100 --warmup 10 --no-cpu-baseline --updates-per-step 1 > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log c5_u1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_learn.py 128 fused > $O/prof.log 2>&1; echo "rocprof rc $?"
