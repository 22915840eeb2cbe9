#!/bin/bash
# async FeAR join: parity tests, then the c5 A/B
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/fasync; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_rollout.py tests/test_actor_ops.py tests/test_maddpg.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -4 $O/pytest.log; [ $s = 0 ] || exit $s
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()})"; }
run c5_fear_async --config c5 --steps 300 --warmup 30 && run c5_sync_fear --config c5 --steps 300 --warmup 30 --sync-fear && \
run c5_fa_eager --config c5 --steps 300 --warmup 30 --obs-lazy && run c3 && \
run c5_learn --config c5 --steps 100 --warmup 20 --updates-per-step 1
