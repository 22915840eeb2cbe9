mkdir -p gpurun_out/v3
echo "== probe" && timeout -k 10 120 ./tools/hbm_probe 537 > gpurun_out/v3/probe.log 2>&1; cat gpurun_out/v3/probe.log
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/v3/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/v3/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > gpurun_out/v3/$tag.log 2>&1; python3 -c "
import json; l=[x for x in open('gpurun_out/v3/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: round(v,4) for k,v in j['kernels_ms'].items()}, j['roofline']['kernel'], round(j['roofline']['achieved']))"; }
EXTRA=""
run split GW_KERNEL=split
run v1 GW_KERNEL=v1
run be2 GW_OBS_BE=2
run be1 GW_OBS_BE=1
run be8 GW_OBS_BE=8
run be4_plain GW_OBS_NT=0
EXTRA="--fear 0"
run split_f0 GW_KERNEL=split
EXTRA="--config c4"
run c4 GW_KERNEL=split
run c4_be2 GW_OBS_BE=2
EXTRA="--config c4f"
run c4f GW_KERNEL=split
