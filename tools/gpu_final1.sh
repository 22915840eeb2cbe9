mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
echo "== bench" && timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log &&
echo "== profile" && bash tools/gpu_profile.sh r1_final --steps 100 --warmup 20 && echo done
