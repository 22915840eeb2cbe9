# round 4 (o): C3 writer flags A/B, 1,000 steps each, same box
O=gpurun_out/r4o; mkdir -p $O
for spec in "base" "GW_OBS_NT=0" "GW_OBS_BE=1" "GW_OBS_BE=4" "base"; do
  if [ $spec = base ]; then e=""; else e=$spec; fi
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --profile-steps 0 > $O/c3_${spec}.log 2>&1 || exit 1
  python tools/bench_line.py $O/c3_${spec}.log "$spec" | head -1
done
