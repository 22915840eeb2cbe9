#!/bin/bash
# fused patch actor: parity tests, c5patch bench (fused vs torch), rocprofv3 stats.  gpurun_out/r3c/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch_actor.py tests/test_gpu_obs_patch.py tests/test_actor_ops.py tests/test_gpu_replay.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --config c5patch --steps 300 --warmup 30 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
timeout -k 10 300 python bench.py --config c5patch --steps 300 --warmup 30 --no-cpu-baseline --updates-per-step 1 > $O/c5patch_u1.log 2>&1 && python tools/bench_line.py $O/c5patch_u1.log c5patch_u1 &&
timeout -k 10 300 python bench.py --config c5patch --steps 100 --warmup 10 --no-cpu-baseline --patch-torch > $O/c5patch_torch.log 2>&1 && python tools/bench_line.py $O/c5patch_torch.log c5patch_torch &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5patch --steps 100 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1; echo "rocprof rc $?"
timeout -k 10 300 python $GRAFT_REPO_ROOT/bench.py --config c4patch --steps 100 --warmup 10 --no-cpu-baseline > $O/c4patch.log 2>&1 && python $GRAFT_REPO_ROOT/tools/bench_line.py $O/c4patch.log c4patch &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4patch --steps 50 --warmup 10 --no-cpu-baseline > $O/prof4.log 2>&1; echo "rocprof4 rc $?"
