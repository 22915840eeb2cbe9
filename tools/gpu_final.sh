#!/bin/bash
# round-end evidence: full GPU suite, smoke, default bench line, c5 rocprofv3 kernel trace
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/final; mkdir -p $O
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] &&
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
echo "== bench" && timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-300 &&
echo "== c5 bench" && timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 30 > $O/bench_c5.log 2>&1 && tail -n 1 $O/bench_c5.log | cut -c1-300 &&
bash tools/gpu_c5prof.sh
