#!/bin/bash
# Graph capture of merged async steps: tests + C2 bench.  gpurun_out/graph2/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/graph2; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
run c2 --config c2 && run c2_eager --config c2 --graph 0 && run c2_g32 --config c2 --graph 32 &&
run c2_d20 --config c2 --steps 20 --warmup 5 && run c1 --config c1 &&
run e16k --envs 16384 && run e16k_eager --envs 16384 --graph 0
