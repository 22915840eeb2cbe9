mkdir -p gpurun_out
echo "== probe" && timeout -k 10 120 ./tools/hbm_probe 537 > gpurun_out/probe.log 2>&1; cat gpurun_out/probe.log
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench fused" && timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1; tail -1 gpurun_out/bench_fused.log | cut -c1-1500
echo "== bench split" && GW_KERNEL=split timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_split.log 2>&1; tail -1 gpurun_out/bench_split.log | cut -c1-1500
for c in c2 c4 c4f; do echo "== bench $c" && timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1; tail -1 gpurun_out/bench_$c.log | cut -c1-1500; done
