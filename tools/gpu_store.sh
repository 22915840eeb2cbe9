#!/bin/bash
# obs store policy A/B (GW_OBS_STORE: 0 nontemporal, 1 sc1, 2 sc0 sc1) + parity of the sc1 path.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/store; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python tools/bench_line.py $O/$n.log $n
}
GW_OBS_STORE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_bench_mode.py tests/test_gpu_obs_bf16.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
for rep in 1 2; do
for st in 0 1 2; do GW_OBS_STORE=$st run c3_s${st}_$rep --steps 1000 --warmup 100 || exit 1; done
done
for st in 0 1 2; do GW_OBS_STORE=$st run bf16_s$st --obs-dtype bf16 || exit 1; done
for st in 0 1; do GW_OBS_STORE=$st run c4_s$st --config c4 --steps 300 --warmup 30 || exit 1; done
for st in 0 1; do GW_OBS_STORE=$st run c5_s$st --config c5 --steps 300 --warmup 30 || exit 1; done
for st in 0 1; do GW_OBS_STORE=$st run c2_s$st --config c2 || exit 1; done
GW_OBS_STORE=1 run d20_s1 --steps 20 --warmup 5 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
GW_OBS_STORE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --no-cpu-baseline --profile-every 0 > $O/prof.log 2>&1 && python tools/gaps.py $O/prof/c3_kernel_trace.csv
