# round 4 (r): the actor workspace derivation at the end of the update graph
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay_desc.py tests/test_gpu_replay.py tests/test_gpu_rollout.py tests/test_maddpg_fused.py tests/test_actor_ops.py > $O/pytest.log 2>&1; s=$?; tail -2 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log c5u1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5u1prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 > $GRAFT_REPO_ROOT/$O/c5u1prof.log 2>&1) || exit 1
echo "== 2-rank gloo C5 rehearsal, ~270 steps: the cap grows only on a growing backlog"
MARLNAV_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c5 --steps 200 --warmup 5 --no-cpu-baseline > $O/c5_gloo2.log 2>&1 && python tools/bench_line.py $O/c5_gloo2.log c5_gloo2 && grep -o '"return_gather[^}]*}' $O/c5_gloo2.log && bash tools/gpu_r4s.sh
