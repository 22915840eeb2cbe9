#!/bin/bash
# Learner change check: the descriptor learner's GPU tests, block stamps, the c5u1 bench line.
T=${1:-r5arow}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O; rm -f $O/stamps.bin
timeout -k 10 600 python -u -m pytest tests/test_gpu_desc_learner.py tests/test_gpu_replay_desc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GW_LEARN_STAMP=$O/stamps.bin timeout -k 10 200 python tools/bench_desc_learn.py 65536 30 > $O/learn.log 2>&1 || { tail -5 $O/learn.log; exit 1; }
tail -3 $O/learn.log
python tools/learn_stamps.py $O/stamps.bin 5 > $O/stamps.txt
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 20 --no-cpu-baseline > $O/c5u1.log 2>&1 || exit 1
python tools/bench_line.py $O/c5u1.log
