#!/bin/bash
# Descriptor learner: its GPU tests, then the learner bench (tools/bench_learn.py) and C5 with one
# update per env step.  Output: gpurun_out/$1/
T=${1:-r5l}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_desc_learner.py tests/test_gpu_replay_desc.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 5 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 20 --no-cpu-baseline > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log
