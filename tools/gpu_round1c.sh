mkdir -p gpurun_out/v2
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/v2/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/v2/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > gpurun_out/v2/$tag.log 2>&1; python3 -c "
import json; l=[x for x in open('gpurun_out/v2/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: round(v,4) for k,v in j['kernels_ms'].items()}, j['roofline']['kernel'], round(j['roofline']['achieved']))"; }
EXTRA=""
run v1 GW_KERNEL=v1
run split GW_KERNEL=split
run fused GW_KERNEL=fused
run split_nt GW_KERNEL=split GW_OBS_NT=1
run split_be4 GW_KERNEL=split GW_OBS_BE=4
run split_be4_nt GW_KERNEL=split GW_OBS_BE=4 GW_OBS_NT=1
EXTRA="--fear 0"
run v1_f0 GW_KERNEL=v1
run split_f0 GW_KERNEL=split
run fused_f0 GW_KERNEL=fused
EXTRA="--config c4"
run c4_split GW_KERNEL=split
run c4_fused GW_KERNEL=fused
run c4_split_nt GW_KERNEL=split GW_OBS_NT=1
