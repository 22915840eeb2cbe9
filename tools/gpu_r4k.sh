# round 4 (k): MODE 4 wave-per-window with batched loads
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python tools/patch_probe.py > $O/probe_m4.log 2>&1 && tail -6 $O/probe_m4.log &&
timeout -k 10 120 python tools/patch_probe.py 65536 11 grid32 stamps > $O/probe_stamps_c5patch.log 2>&1 && tail -3 $O/probe_stamps_c5patch.log &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
timeout -k 10 300 python bench.py --config c4patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c4patch.log 2>&1 && python tools/bench_line.py $O/c4patch.log c4patch &&
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_driver_$i.log 2>&1 || exit 1; python tools/bench_line.py $O/c3_driver_$i.log c3_driver_$i; grep -o '"host_first_steps_us": \[[^]]*\]' $O/c3_driver_$i.log; done
timeout -k 10 150 python tools/bench_learn.py 128 > $O/learn.log 2>&1 && tail -2 $O/learn.log
