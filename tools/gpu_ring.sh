#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ring; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }; python tools/bench_line.py $O/$n.log $n; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_bench_mode.py tests/test_gpu_rollout.py tests/test_gpu_replay.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
for rep in 1 2; do
run c3_ring2_$rep --steps 1000 --warmup 100 && run c3_ring1_$rep --steps 1000 --warmup 100 --obs-ring 1 || exit 1
done
run d20 --steps 20 --warmup 5 && run c5 --config c5 --steps 300 --warmup 30 && run bf16 --obs-dtype bf16 &&
run c4 --config c4 --steps 300 --warmup 30 && run c4f --config c4f --steps 300 --warmup 30 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --steps 300 --warmup 30 --no-cpu-baseline --profile-every 0 > $O/prof.log 2>&1 && python tools/gaps.py $O/prof/c3_kernel_trace.csv &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof5 -o c5 -- python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof5.log 2>&1 && grep -E "tick|act_kernel" $O/prof5/c5_kernel_stats.csv | cut -c1-150
