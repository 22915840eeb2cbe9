# round 4 (n): descriptor copy inside the step kernels; C5 + update; rooflines for c5patch and c2
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay_desc.py tests/test_gpu_replay.py tests/test_gpu_rollout.py tests/test_gpu_rollout_graph.py tests/test_gpu_bench_c5_c2.py > $O/pytest.log 2>&1; s=$?; tail -2 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5u1.log 2>&1 && python tools/bench_line.py $O/c5u1.log c5u1 &&
bash tools/gpu_roofline.sh r4_end2 c5patch c2
