mkdir -p gpurun_out/v4; rm -f gpurun_out/v4/*.log
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/v4/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/v4/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > gpurun_out/v4/$tag.log 2>&1; python3 -c "
import json; l=[x for x in open('gpurun_out/v4/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: round(v,4) for k,v in j['kernels_ms'].items()}, j['roofline']['kernel'], round(j['roofline']['achieved']))"; }
EXTRA=""
run ch4 GW_CHUNKS=4
run ch1 GW_CHUNKS=1
run ch2 GW_CHUNKS=2
run ch8 GW_CHUNKS=8
run ch4_be8 GW_CHUNKS=4 GW_OBS_BE=8
run ch4_plain GW_CHUNKS=4 GW_OBS_NT=0
run ch1_be2 GW_CHUNKS=1 GW_OBS_BE=2
run ch4_be2 GW_CHUNKS=4 GW_OBS_BE=2
run ch3 GW_CHUNKS=3
EXTRA="--config c4"
run c4_ch4 GW_CHUNKS=4
run c4_ch1 GW_CHUNKS=1
EXTRA="--config c4f"
run c4f_ch4 GW_CHUNKS=4
