R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pasync; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_patch_actor.py tests/test_gpu_patch_cnn.py tests/test_gpu_obs_patch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || exit $s
for c in c4patch c5patch; do for i in 1 2; do
  GW_PATCH_ASYNC=0 timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline > $O/${c}_sync_$i.log 2>&1 && python tools/bench_line.py $O/${c}_sync_$i.log ${c}_sync_$i || exit 1
  timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline > $O/${c}_async_$i.log 2>&1 && python tools/bench_line.py $O/${c}_async_$i.log ${c}_async_$i || exit 1
done; done
