#!/bin/bash
# bf16x3 layer-2 actor (GW_ACT_V=4): parity vs torch fp32, isolated timing, c5
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/act4; mkdir -p $O
GW_ACT_V=4 timeout -k 10 200 python -u -m pytest tests/test_actor_ops.py tests/test_gpu_async_obs.py -x -q --timeout 120 --timeout-method thread > $O/t4.log 2>&1; s=$?; tail -n 3 $O/t4.log; [ $s = 0 ] || exit $s
for v in 2 4; do GW_ACT_V=$v timeout -k 10 100 python tools/act_ab.py grid32 65536 200 > $O/ab$v.log 2>&1 || exit 1; echo v$v; head -4 $O/ab$v.log | tail -n 3; grep eager $O/ab$v.log; done
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
C="--config c5 --steps 300 --warmup 30"
GW_ACT_V=2 run c5_v2 $C && GW_ACT_V=4 run c5_v4 $C && GW_ACT_V=4 run c5_v4_fa $C --fear-async
