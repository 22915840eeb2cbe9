#!/bin/bash
# world update with 32 envs per wave (2 latency chains per SIMD): full GPU suite, then the bench lines
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/half; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 1 $O/pytest.log; [ $s = 0 ] || { grep -E "^E |FAIL" $O/pytest.log | head; exit $s; }
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', 'step', round(k['step_kernel']*1e3,1), 'obs', round(k['obs_kernel']*1e3,1), 'fear', round(k['fear_kernel']*1e3,1))"; }
run c3 && run c3b --obs-dtype bf16 && run c5 --config c5 --steps 300 --warmup 30 && run c5b --config c5 --steps 300 --warmup 30 --obs-dtype bf16 && \
run c2 --config c2 && run c4 --config c4 && run c4f --config c4f && run c3_sync --sync-obs
