# round 4 (w): launches recorded from an eager update (ordinary allocator buffers) vs the graph replay
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay_desc.py tests/test_gpu_rollout.py tests/test_maddpg_fused.py tests/test_actor_ops.py tests/test_maddpg.py > $O/pytest.log 2>&1; s=$?; tail -2 $O/pytest.log; [ $s = 0 ] || exit $s
for m in graph launches; do
  extra=""; [ $m = launches ] && extra="--learn-launches"
  timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline $extra > $O/c5u1_$m.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5u1_$m.log "c5u1 $m" | head -1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/launchprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 --learn-launches > $GRAFT_REPO_ROOT/$O/launchprof.log 2>&1) || exit 1
