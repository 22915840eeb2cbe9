# cost of the per-kernel timing events: profile every step / every 8th / never
mkdir -p gpurun_out/v9; rm -f gpurun_out/v9/*.log
B="python bench.py --steps 400 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > gpurun_out/v9/$tag.log 2>&1 || return 1; python3 -c "
import json; l=[x for x in open('gpurun_out/v9/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()})" || tail -3 gpurun_out/v9/$tag.log; }
EXTRA="--profile-every 1" && run p1 GW_KERNEL=split && EXTRA="--profile-every 8" && run p8 GW_KERNEL=split && \
EXTRA="--profile-every 0" && run p0 GW_KERNEL=split && EXTRA="--profile-every 8" && run d3p8 GW_KERNEL=defer GW_DEFER=3 && \
EXTRA="--profile-every 0" && run d3p0 GW_KERNEL=defer GW_DEFER=3 && run d0p0 GW_KERNEL=defer GW_DEFER=0 && \
EXTRA="--profile-every 8 --config c4f" && run c4f_split GW_KERNEL=split && run c4f_d3 GW_KERNEL=defer GW_DEFER=3
