#!/bin/bash
# C2 (grid32, 4,096 envs, FeAR off) chain: parity tests of the FeAR-off step paths, two bench runs,
# rocprofv3 kernel stats of the step-only and merged kernels.  Output: gpurun_out/$1/
T=${1:-c2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_c5_c2.py tests/test_gpu_graph.py tests/test_gpu_async_obs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_$i.log 2>&1 && python tools/bench_line.py $O/c2_$i.log c2_$i || exit 1
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof$m -o run --output-format csv -- python3 $ROOT/tools/c2_probe.py $m > $O/prof$m.log 2>&1 || exit 1
  f=$(find $O/prof$m -name '*kernel_stats.csv' | head -n 1); head -n 3 "$f"
done
