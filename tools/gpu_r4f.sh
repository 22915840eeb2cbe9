# round 4 (f): learner staging loads prefetched (l1 / grads / gemv16); window writer 64 envs per block (A/B)
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_maddpg_fused.py tests/test_maddpg.py tests/test_gpu_obs_patch.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
GW_PATCH_PB=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py tests/test_gpu_patch_actor.py > $O/pytest_pb64.log 2>&1; s=$?; tail -3 $O/pytest_pb64.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/bench_learn.py 128 > $O/learn.log 2>&1 && tail -1 $O/learn.log &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/learnprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_learn.py 128 > $GRAFT_REPO_ROOT/$O/learnprof.log 2>&1) &&
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log c5u1 &&
timeout -k 10 120 python tools/patch_probe.py > $O/probe_pb32.log 2>&1 && tail -6 $O/probe_pb32.log &&
GW_PATCH_PB=64 timeout -k 10 120 python tools/patch_probe.py > $O/probe_pb64.log 2>&1 && tail -6 $O/probe_pb64.log &&
GW_PATCH_PB=64 timeout -k 10 120 python tools/patch_probe.py 65536 11 grid32 stamps > $O/probe_stamps_c5patch_pb64.log 2>&1 &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
GW_PATCH_PB=64 timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch_pb64.log 2>&1 && python tools/bench_line.py $O/c5patch_pb64.log c5patch_pb64 &&
GW_PATCH_PB=64 timeout -k 10 300 python bench.py --config c4patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c4patch_pb64.log 2>&1 && python tools/bench_line.py $O/c4patch_pb64.log c4patch_pb64
