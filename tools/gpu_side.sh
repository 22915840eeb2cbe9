#!/bin/bash
# statistics reduction on a side stream (Rollout side_tick): rollout tests, C5 A/B
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/side; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_async_obs.py tests/test_actor_ops.py tests/test_gpu_obs_bf16.py tests/test_maddpg.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; s=$?; tail -n 1 $O/t.log; [ $s = 0 ] || { grep -E "^E |FAIL" $O/t.log | head; exit $s; }
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']; print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G')"; }
C="--config c5 --steps 300 --warmup 30"
run c5_side $C && run c5b_side $C --obs-dtype bf16 && run c5_side_learn --config c5 --steps 100 --warmup 20 --updates-per-step 1
