mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log &&
echo "== pytest gpu" && timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; 
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench" && timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 8 > gpurun_out/bench.log 2>&1; tail -3 gpurun_out/bench.log
