#!/bin/bash
# stream-priority A/B of the async obs pipeline, then the rocprofv3 evidence of the new default
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prio; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()}, round(j['roofline']['step_level_GBps']))"; }
run c3_default && GW_OBS_PRIO=hi run c3_obshi && GW_OBS_BE=2 run c3_be2 && GW_OBS_BE=8 run c3_be8 && GW_OBS_NT=0 run c3_plain && \
GW_OBS_PRIO=hi run c4f_obshi --config c4f && run c4f_default --config c4f && \
./tools/gpu_profile.sh r1_c3_async --steps 200 --warmup 20
