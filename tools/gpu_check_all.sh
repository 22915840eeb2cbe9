#!/bin/bash
# Full GPU check of the current tree: gpu tests, smoke(), default bench line.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/check; mkdir -p $O
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -5 $O/pytest.log; [ $s = 0 ] &&
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log &&
echo "== bench" && timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
