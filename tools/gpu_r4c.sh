# round 4 (c): descriptor replay ring + 4-wave actor blocks; C5 with one update per step
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay_desc.py tests/test_actor_ops.py tests/test_gpu_rollout.py tests/test_gpu_rollout_graph.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log c5u1 &&
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline --dense-learn > $O/c5u1_dense.log 2>&1 && python tools/bench_line.py $O/c5u1_dense.log c5u1_dense &&
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_200.log 2>&1 && python tools/bench_line.py $O/c2_200.log c2_200 &&
GW_ACT_WAVES=16 timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_200_w16.log 2>&1 && python tools/bench_line.py $O/c2_200_w16.log c2_200_w16 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c5u1prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 > $GRAFT_REPO_ROOT/$O/c5u1prof.log 2>&1)
