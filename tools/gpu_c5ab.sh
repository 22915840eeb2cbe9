#!/bin/bash
# C5 pipeline variants with the current actor: lazy (default) / eager obs, FeAR joined / overlapped
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c5ab; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
C="--config c5 --steps 300 --warmup 30"
run lazy $C && run eager $C --obs-eager && run lazy_fa $C --fear-async && run eager_fa $C --obs-eager --fear-async && run sync $C --sync-obs && run lazy_p0 $C --profile-every 0
