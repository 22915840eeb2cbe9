#!/bin/bash
# actor variants (GW_ACT_V) x async FeAR join on the c5 rollout
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/act2; mkdir -p $O
GW_ACT_V=2 timeout -k 10 200 python -u -m pytest tests/test_actor_ops.py tests/test_gpu_async_obs.py -x -q --timeout 120 --timeout-method thread > $O/t2.log 2>&1; s=$?; tail -n 1 $O/t2.log; [ $s = 0 ] || exit $s
for v in 0 2; do GW_ACT_V=$v timeout -k 10 100 python tools/act_ab.py grid32 65536 200 > $O/ab$v.log 2>&1 || exit 1; head -3 $O/ab$v.log | tail -n 2; grep eager $O/ab$v.log; done
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()})"; }
C="--config c5 --steps 300 --warmup 30"
GW_ACT_V=0 run v0_fa $C && GW_ACT_V=0 run v0_sf $C --sync-fear && GW_ACT_V=2 run v2_fa $C && GW_ACT_V=2 run v2_sf $C --sync-fear && GW_ACT_V=2 run v2_fa_sync $C --sync-obs
