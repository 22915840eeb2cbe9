#!/bin/bash
# Auto-selected merged path for small batches: full GPU suite, then the merged / defer crossover
# over envs per GPU (C3 shape, FeAR on) and C2.  gpurun_out/merged2/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/merged2; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
for e in 2048 4096 8192 16384 32768; do
  GW_KERNEL=merged run m_$e --envs $e --steps 500 --warmup 50 &&
  GW_KERNEL=defer run d_$e --envs $e --steps 500 --warmup 50 --obs-eager &&
  GW_KERNEL=defer run ds_$e --envs $e --steps 500 --warmup 50 --sync-obs || exit 1
done
run c2 --config c2 &&
GW_KERNEL=merged run c2_m_nograph --config c2 --graph 0 &&
run c1 --config c1 &&
run c3 --steps 1000 --warmup 100
