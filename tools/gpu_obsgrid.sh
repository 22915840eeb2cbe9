#!/bin/bash
# capped (grid-stride) obs writer: parity, then C3 / C5 A/B over the grid cap
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/obsgrid; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "defer" -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; s=$?; tail -n 1 $O/t.log; [ $s = 0 ] || exit $s
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
for g in 0 256 512 1024 2048; do GW_OBS_GRID=$g run c3_g$g || exit 1; done
C="--config c5 --steps 300 --warmup 30"
for g in 0 512 1024; do GW_ACT_V=2 GW_OBS_GRID=$g run c5v2_sf_g$g $C --sync-fear && GW_ACT_V=2 GW_OBS_GRID=$g run c5v2_fa_g$g $C || exit 1; done
GW_ACT_V=2 GW_OBS_GRID=512 run c5v2_fa_eager_g512 $C --obs-eager
