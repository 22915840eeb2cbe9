#!/bin/bash
# Round-2 final check: full GPU suite, smoke, the default bench line (driver command and long run).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/final_r2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 && python tools/bench_line.py $O/bench_driver.log driver &&
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 && python tools/bench_line.py $O/bench_default.log default &&
tail -n 1 $O/bench_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['cpu_baseline'])"
