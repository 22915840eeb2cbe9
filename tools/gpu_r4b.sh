O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_return_compact.py tests/test_gpu_replay_desc.py tests/test_gpu_obs_patch.py tests/test_gpu_checkpoint_eval.py tests/test_gpu_rollout_graph.py tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py tests/test_gpu_cnn_actor.py tests/test_actor_ops.py tests/test_gpu_rollout.py tests/test_gpu_async_obs.py tests/test_gpu_dist.py tests/test_gpu_return_compact.py tests/test_gpu_gather_pack.py tests/test_maddpg_dp.py tests/test_maddpg_fused.py tests/test_maddpg.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/bench_learn.py 128 > $O/learn.log 2>&1 && tail -2 $O/learn.log &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/learnprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_learn.py 128 > $GRAFT_REPO_ROOT/$O/learnprof.log 2>&1) || exit 1
for m in 0 3; do GW_PATCH_MODE=$m timeout -k 10 120 python tools/patch_probe.py > $O/probe_m$m.log 2>&1 || exit 1; done
timeout -k 10 120 python tools/patch_probe.py 65536 16 grid64_n8 stamps > $O/probe_stamps_c4patch.log 2>&1 || exit 1
timeout -k 10 120 python tools/patch_probe.py 65536 11 grid32 stamps > $O/probe_stamps_c5patch.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.log 2>&1 && python tools/bench_line.py $O/c2.log c2 &&
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_200.log 2>&1 && python tools/bench_line.py $O/c2_200.log c2_200 &&
GW_ACT_WAVES=16 timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_200_w16.log 2>&1 && python tools/bench_line.py $O/c2_200_w16.log c2_200_w16 &&
timeout -k 10 300 python bench.py --config c2env --steps 200 --warmup 20 --no-cpu-baseline > $O/c2env.log 2>&1 && python tools/bench_line.py $O/c2env.log c2env &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 && python tools/bench_line.py $O/c5.log c5
echo "== C3 CU split A/B (1000 steps)"
for spec in "0 first" "48 first" "64 first" "96 first" "64 strided" "0 first" "48 strided" "32 strided"; do
  set -- $spec
  if [ $1 = 0 ]; then unset GW_CU_SPLIT; else export GW_CU_SPLIT=$1; fi
  export GW_CU_PATTERN=$2
  timeout -k 10 200 python bench.py --no-cpu-baseline --profile-steps 0 > $O/c3_split_$1_$2.log 2>&1 || exit 1
  python tools/bench_line.py $O/c3_split_$1_$2.log "split $1 $2" | head -1
done
unset GW_CU_SPLIT GW_CU_PATTERN
echo "== 2-rank gloo C5 rehearsal (one GPU): packed return gather bytes per rank per step"
MARLNAV_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_gloo2.log 2>&1 && python tools/bench_line.py $O/c5_gloo2.log c5_gloo2
