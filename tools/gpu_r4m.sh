# round 4 (m): MODE 4 wave copy restored (odd P), MODE 2 for P % 4 == 0; 64 envs per block A/B
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py > $O/pytest.log 2>&1; s=$?; tail -2 $O/pytest.log; [ $s = 0 ] || exit $s
GW_PATCH_PB=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py > $O/pytest_pb64.log 2>&1; s=$?; tail -2 $O/pytest_pb64.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/patch_probe.py > $O/probe.log 2>&1 && tail -6 $O/probe.log &&
GW_PATCH_PB=64 timeout -k 10 120 python tools/patch_probe.py > $O/probe_pb64.log 2>&1 && tail -6 $O/probe_pb64.log &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
GW_PATCH_PB=64 timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch_pb64.log 2>&1 && python tools/bench_line.py $O/c5patch_pb64.log c5patch_pb64 &&
timeout -k 10 300 python bench.py --config c4patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c4patch.log 2>&1 && python tools/bench_line.py $O/c4patch.log c4patch
