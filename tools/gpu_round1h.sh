# defer-mode check: GPU suite + A/B of split vs defer at C3 and C4f
mkdir -p gpurun_out/v7; rm -f gpurun_out/v7/*.log
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/v7/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/v7/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > gpurun_out/v7/$tag.log 2>&1 || return 1; python3 -c "
import json; l=[x for x in open('gpurun_out/v7/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()})" || tail -3 gpurun_out/v7/$tag.log; }
EXTRA=""; run def GW_KERNEL=split && run defer GW_KERNEL=defer && \
EXTRA="--config c4f"; run c4f GW_KERNEL=split && run c4f_defer GW_KERNEL=defer
