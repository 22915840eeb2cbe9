#!/bin/bash
# C5 default (eager writer in 2 launches) vs the round-2 lazy default: chunked-writer parity
# tests, repeated bench lines, a kernel trace of the default.  gpurun_out/c5def/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c5def; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_async_obs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chunked" > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
for rep in 1 2 3; do
run c5_def_$rep --config c5 --steps 300 --warmup 30 &&
GW_OBS_CHUNKS=1 run c5_lazy1_$rep --config c5 --steps 300 --warmup 30 --obs-lazy || exit 1
done
run c5_d20 --config c5 --steps 20 --warmup 5 &&
run c5_long --config c5 --steps 1000 --warmup 100 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python bench.py --no-cpu-baseline --config c5 --steps 300 --warmup 30 --profile-every 0 > $O/prof.log 2>&1 && python tools/gaps.py $O/prof/c5_kernel_trace.csv > $O/gaps.txt 2>&1; tail -3 $O/prof.log
