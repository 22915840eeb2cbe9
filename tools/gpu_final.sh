#!/bin/bash
# round-end evidence: full GPU suite, smoke, bench lines (C3 default with cpu_baseline, C3 bf16,
# C5), then the rocprofv3 trace + FETCH/WRITE passes of the C3 default (tools/gpu_profile.sh)
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/final; mkdir -p $O
echo "== pytest -m gpu" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 1 $O/pytest.log; [ $s = 0 ] || { grep -E "^E |FAIL" $O/pytest.log | head; exit $s; }
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
echo "== bench" && timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-200 &&
echo "== bench bf16" && timeout -k 10 300 python bench.py --obs-dtype bf16 --no-cpu-baseline > $O/bench_bf16.log 2>&1 &&
echo "== bench c5" && timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 30 --no-cpu-baseline > $O/bench_c5.log 2>&1 &&
bash tools/gpu_profile.sh r1_c3_final2 --steps 200 --warmup 20
