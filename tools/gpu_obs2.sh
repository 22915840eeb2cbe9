#!/bin/bash
# two alternating obs streams + double-buffered bench outputs vs one stream / one buffer
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/obs2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; s=$?; tail -n 1 $O/t.log; [ $s = 0 ] || exit $s
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
run c3 && run c3_1buf --obs-single-buffer && GW_OBS_STREAMS=1 run c3_1stream && GW_OBS_STREAMS=1 run c3_1s1b --obs-single-buffer && \
run c4f --config c4f && run c4 --config c4 && run c2 --config c2 && run c5 --config c5 --steps 300 --warmup 30
