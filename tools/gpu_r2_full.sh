#!/bin/bash
# Round-2 state check: full GPU suite, smoke, the bench configs and a rocprofv3 kernel trace
# of the default bench command.  Output under gpurun_out/r2full/.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r2full; mkdir -p $O
echo "== full suite" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
echo "== bench c3" && timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-500 &&
echo "== bench c3 driver-size" && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_20.log 2>&1 && tail -n 1 $O/bench_20.log | cut -c1-300 &&
echo "== bench c2" && timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > $O/bench_c2.log 2>&1 && tail -n 1 $O/bench_c2.log | cut -c1-300 &&
echo "== bench c5" && timeout -k 10 300 python bench.py --config c5 --steps 300 --warmup 30 --no-cpu-baseline > $O/bench_c5.log 2>&1 && tail -n 1 $O/bench_c5.log | cut -c1-300 &&
echo "== bench c4cnn" && timeout -k 10 300 python bench.py --config c4cnn --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_c4cnn.log 2>&1 && tail -n 1 $O/bench_c4cnn.log | cut -c1-300 &&
echo "== bench c3 bf16" && timeout -k 10 300 python bench.py --obs-dtype bf16 --no-cpu-baseline > $O/bench_bf16.log 2>&1 && tail -n 1 $O/bench_bf16.log | cut -c1-300 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
echo "== rocprof c3" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $O/prof.log 2>&1 && tail -n 1 $O/prof.log | cut -c1-300
