#!/bin/bash
# Round-5 checks: the learner's and the window-graph tests, the learner profile, c5u1 / c4patch / c5patch lines.
T=${1:-r5b}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$T; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_desc_learner.py tests/test_maddpg_fused.py tests/test_gpu_rollout_graph.py tests/test_gpu_patch_cnn.py tests/test_gpu_obs_patch.py -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 4 $O/pytest.log; [ $s = 0 ] || exit $s
bash $GRAFT_REPO_ROOT/tools/gpu_r5_lprof.sh $T || exit 1
for c in "c5 --updates-per-step 1 --steps 100 --warmup 20" "c4patch --steps 200 --warmup 20" "c5patch --steps 200 --warmup 20" "c3 --steps 20 --warmup 5"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$n.log 2>&1 || exit 1
  python tools/bench_line.py $O/bench_$n.log
done
