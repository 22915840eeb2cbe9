#!/bin/bash
# lossless bf16 obs: parity vs the float32 path, then the bench lines (reported separately)
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/bf16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_obs_bf16.py tests/test_gpu_async_obs.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; s=$?; tail -n 1 $O/t.log; [ $s = 0 ] || { grep -E "^E |FAIL" $O/t.log | head; exit $s; }
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; r=j['roofline']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1), 'obsGB/s', round(r['achieved']))"; }
run c3_bf16 --obs-dtype bf16 && GW_OBS_BE=16 run c3_bf16_be16 --obs-dtype bf16 && run c3_f32 && run c4f_bf16 --config c4f --obs-dtype bf16 && run c4_bf16 --config c4 --obs-dtype bf16 && \
GW_OBS_BE=8 run c4_bf16_be8 --config c4 --obs-dtype bf16 && run c5_bf16 --config c5 --steps 300 --warmup 30 --obs-dtype bf16 && run c2_bf16 --config c2 --obs-dtype bf16
