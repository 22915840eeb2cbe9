# round 4 (h): tails back to global operands (LDS staging measured slower), actor prepare loads batched,
# sample microbench (dense vs descriptor rows), C5 + one update per step
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_maddpg_fused.py tests/test_maddpg.py tests/test_actor_ops.py tests/test_gpu_replay_desc.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/bench_learn.py 128 > $O/learn.log 2>&1 && tail -1 $O/learn.log &&
timeout -k 10 120 python tools/bench_sample.py > $O/sample.log 2>&1 && tail -4 $O/sample.log &&
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log c5u1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5u1prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 > $GRAFT_REPO_ROOT/$O/c5u1prof.log 2>&1) &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/learnprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_learn.py 128 > $GRAFT_REPO_ROOT/$O/learnprof.log 2>&1)
GW_PATCH_MODE=9 timeout -k 10 120 python tools/patch_probe.py > $O/probe_floor.log 2>&1 && tail -6 $O/probe_floor.log
