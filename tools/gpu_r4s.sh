# round 4 (s): obs streams at low priority (GW_OBS_PRIO=lo) A/B on c5u1, c5, c3
O=gpurun_out/r4s; mkdir -p $O
for prio in normal lo; do
  if [ $prio = lo ]; then export GW_OBS_PRIO=lo; else unset GW_OBS_PRIO; fi
  timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 10 --no-cpu-baseline > $O/c5u1_$prio.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5u1_$prio.log "c5u1 $prio" | head -1
  timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 10 --no-cpu-baseline > $O/c5_$prio.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5_$prio.log "c5 $prio" | head -1
  timeout -k 10 300 python bench.py --steps 1000 --warmup 20 --no-cpu-baseline > $O/c3_$prio.log 2>&1 || exit 1
  python tools/bench_line.py $O/c3_$prio.log "c3 $prio" | head -1
done
