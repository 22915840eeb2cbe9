#!/bin/bash
# kernel path A/B under the async pipeline: defer (world update, then fear_v2) vs split (FeAR inline)
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/split; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
C5="--config c5 --steps 300 --warmup 30"
GW_KERNEL=split run c3_split && GW_KERNEL=split run c3b_split --obs-dtype bf16 && run c3b_defer --obs-dtype bf16 && \
GW_KERNEL=split run c5_split $C5 && GW_KERNEL=split run c5b_split $C5 --obs-dtype bf16 && run c5b_defer $C5 --obs-dtype bf16 && \
GW_KERNEL=split GW_FEAR_BE=wide run c3_split_wide && GW_FEAR_BE=wide run c3b_defer_wide --obs-dtype bf16 && GW_KERNEL=split run c4f_split --config c4f
