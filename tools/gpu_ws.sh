#!/bin/bash
# async chain on the caller's stream vs on the aux stream (GW_ASYNC_AUX=1)
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ws; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; s=$?; tail -n 1 $O/t.log; [ $s = 0 ] || exit $s
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
C="--config c5 --steps 300 --warmup 30"
run c3_s && GW_ASYNC_AUX=1 run c3_aux && run c3_s_p0 --profile-every 0 && GW_ASYNC_AUX=1 run c3_aux_p0 --profile-every 0 && \
run c5_s $C && GW_ASYNC_AUX=1 run c5_aux $C && run c4f_s --config c4f && run c2_s --config c2 && GW_ASYNC_AUX=1 run c2_aux --config c2
