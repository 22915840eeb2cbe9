O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py tests/test_gpu_checkpoint_eval.py tests/test_gpu_rollout_graph.py tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py tests/test_gpu_async_obs.py > $O/pytest.log 2>&1; s=$?; tail -3 $O/pytest.log; [ $s = 0 ] || exit $s
for m in 0 3; do GW_PATCH_MODE=$m timeout -k 10 120 python tools/patch_probe.py > $O/probe_m$m.log 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.log 2>&1 && python tools/bench_line.py $O/c2.log c2 &&
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_200.log 2>&1 && python tools/bench_line.py $O/c2_200.log c2_200 &&
timeout -k 10 300 python bench.py --config c2env --steps 200 --warmup 20 --no-cpu-baseline > $O/c2env.log 2>&1 && python tools/bench_line.py $O/c2env.log c2env &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5.log 2>&1 && python tools/bench_line.py $O/c5.log c5
