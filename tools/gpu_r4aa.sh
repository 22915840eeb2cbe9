# round 4 (aa): c5patch with the window writer on a side stream beside the next actor (GW_PATCH_ASYNC=1) vs default
O=gpurun_out/r4aa; mkdir -p $O
for m in default 1; do
  if [ $m = 1 ]; then export GW_PATCH_ASYNC=1; else unset GW_PATCH_ASYNC; fi
  timeout -k 10 300 python bench.py --config c5patch --steps 200 --warmup 10 --no-cpu-baseline > $O/c5patch_$m.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5patch_$m.log "c5patch async=$m" | head -2
done
