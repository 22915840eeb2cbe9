# round 4 (j): window writer MODE 4 (table copy + patch stores): parity tests, probes, rollouts
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/patch_probe.py > $O/probe_m4.log 2>&1 && tail -6 $O/probe_m4.log &&
GW_PATCH_TABLE=0 timeout -k 10 120 python tools/patch_probe.py > $O/probe_notbl.log 2>&1 && tail -6 $O/probe_notbl.log &&
timeout -k 10 120 python tools/patch_probe.py 65536 11 grid32 stamps > $O/probe_stamps_c5patch.log 2>&1 && tail -3 $O/probe_stamps_c5patch.log &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
timeout -k 10 300 python bench.py --config c4patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c4patch.log 2>&1 && python tools/bench_line.py $O/c4patch.log c4patch
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/c3trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-steps 0 > $GRAFT_REPO_ROOT/$O/c3trace.log 2>&1) && python tools/run_span.py $O/c3trace/run_kernel_trace.csv 20
