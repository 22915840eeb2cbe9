# round 4 (z): window writer MODE 5 (table rows as aligned float4 runs, loads batched) vs the default
O=gpurun_out/r4z; mkdir -p $O
GW_PATCH_MODE=5 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_obs_patch.py tests/test_gpu_patch_actor.py > $O/pytest_mode5.log 2>&1; s=$?; tail -2 $O/pytest_mode5.log; [ $s = 0 ] || exit $s
timeout -k 10 200 python tools/patch_probe.py > $O/probe_default.log 2>&1 || exit 1
GW_PATCH_MODE=5 timeout -k 10 200 python tools/patch_probe.py > $O/probe_mode5.log 2>&1 || exit 1
echo "== default"; cat $O/probe_default.log | grep -v amdgpu.ids
echo "== MODE 5"; cat $O/probe_mode5.log | grep -v amdgpu.ids
for m in default 5; do
  if [ $m = 5 ]; then export GW_PATCH_MODE=5; else unset GW_PATCH_MODE; fi
  timeout -k 10 300 python bench.py --config c5patch --steps 200 --warmup 10 --no-cpu-baseline > $O/c5patch_$m.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5patch_$m.log "c5patch $m" | head -2
done
