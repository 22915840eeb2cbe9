#!/bin/bash
# End-of-milestone check: full GPU suite, smoke, the driver's bench command, the default long run,
# then rocprofv3 (kernel trace + FETCH_SIZE / WRITE_SIZE passes) of the driver's command.
# Usage: tools/gpu_final.sh TAG   -> gpurun_out/TAG/
T=${1:-final}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 && python tools/bench_line.py $O/bench_driver.log driver &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.log 2>&1 && python tools/bench_line.py $O/bench_default.log default &&
bash tools/gpu_profile.sh $T --gpus 1 --steps 20 --warmup 5 > $O/profile.log 2>&1; echo "profile rc $?"
