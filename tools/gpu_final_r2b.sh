#!/bin/bash
# Round-2 end check after the learner changes: full GPU suite, smoke, driver-size and default
# bench lines, then the §8f next rows (tools/bench_next.py).  gpurun_out/final_r2b/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/final_r2b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 && python tools/bench_line.py $O/bench_driver.log driver &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.log 2>&1 && python tools/bench_line.py $O/bench_default.log default &&
timeout -k 10 300 python tools/bench_next.py > $O/next.log 2>&1 && grep row $O/next.log
