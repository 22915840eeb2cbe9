#!/bin/bash
# Round-2 check: the new / changed GPU tests first, then the full suite, smoke and bench A/B
# (return gather on / off) for C3 and C5.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r2; mkdir -p $O
echo "== new tests" &&
timeout -k 10 600 python -u -m pytest tests/test_maddpg.py tests/test_gpu_dist.py tests/test_gpu_bench_mode.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1; s=$?; tail -n 3 $O/pytest_new.log; [ $s = 0 ] || exit $s
echo "== full suite" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
echo "== bench c3" && timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-400 &&
echo "== bench c3 driver-size" && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20.log 2>&1 && tail -n 1 $O/bench_20.log | cut -c1-300 &&
echo "== bench c3 no gather" && timeout -k 10 300 python bench.py --no-gather --no-cpu-baseline > $O/bench_ng.log 2>&1 && tail -n 1 $O/bench_ng.log | cut -c1-300 &&
echo "== bench c5" && timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 30 --no-cpu-baseline > $O/bench_c5.log 2>&1 && tail -n 1 $O/bench_c5.log | cut -c1-300 &&
echo "== bench c5 no gather" && timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 30 --no-cpu-baseline --no-gather > $O/bench_c5ng.log 2>&1 && tail -n 1 $O/bench_c5ng.log | cut -c1-300
