#!/bin/bash
# Full check: GPU suite, smoke, driver-size bench line.  Output: gpurun_out/$1/
T=${1:-check}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 && tail -c 600 $O/bench_driver.log
