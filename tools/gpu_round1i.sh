# defer-mode ordering A/B (C3 and C4f)
mkdir -p gpurun_out/v8; rm -f gpurun_out/v8/*.log
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > gpurun_out/v8/$tag.log 2>&1 || return 1; python3 -c "
import json; l=[x for x in open('gpurun_out/v8/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()})" || tail -3 gpurun_out/v8/$tag.log; }
EXTRA="" && run split GW_KERNEL=split && run d0 GW_KERNEL=defer GW_DEFER=0 && run d1 GW_KERNEL=defer GW_DEFER=1 && \
run d2 GW_KERNEL=defer GW_DEFER=2 && run d3 GW_KERNEL=defer GW_DEFER=3 && \
EXTRA="--config c4f" && run c4f_d0 GW_KERNEL=defer GW_DEFER=0 && run c4f_d2 GW_KERNEL=defer GW_DEFER=2 && run c4f_d3 GW_KERNEL=defer GW_DEFER=3
