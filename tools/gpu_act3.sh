#!/bin/bash
# ping-pong actor (GW_ACT_V=3) vs the 16-wave default: parity, isolated timing, c5
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/act3; mkdir -p $O
GW_ACT_V=3 timeout -k 10 200 python -u -m pytest tests/test_actor_ops.py tests/test_gpu_async_obs.py -x -q --timeout 120 --timeout-method thread > $O/t3.log 2>&1; s=$?; tail -n 1 $O/t3.log; [ $s = 0 ] || exit $s
for v in 2 3; do GW_ACT_V=$v timeout -k 10 100 python tools/act_ab.py grid32 65536 200 > $O/ab$v.log 2>&1 || exit 1; echo v$v; head -9 $O/ab$v.log | tail -n 8; grep eager $O/ab$v.log; done
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
C="--config c5 --steps 300 --warmup 30"
GW_ACT_V=2 run c5_v2 $C && GW_ACT_V=3 run c5_v3 $C && GW_ACT_V=3 run c5_v3_fa $C --fear-async && run c3
