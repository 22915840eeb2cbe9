# round 4 (x): the driver's bench invocations on the final code (default flags; --steps 20 --warmup 5)
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || exit 1
tail -1 $O/bench_default.log | cut -c1-400
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_20.log 2>&1 || exit 1
python tools/bench_line.py $O/bench_20.log "c3 driver size" | head -1
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline > $O/c5u1.log 2>&1 || exit 1
python tools/bench_line.py $O/c5u1.log "c5u1 default (launches)" | head -1
