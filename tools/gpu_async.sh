#!/bin/bash
# async-obs pipeline: parity tests, then A/B of the bench (c3, c4f, c5) sync vs async
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/async; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_async_obs.py tests/test_gpu_rollout.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -4 $O/pytest.log; [ $s = 0 ] || exit $s
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), round(j['value']/1e9,3), 'G', {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items()}, round(j['roofline']['step_level_GBps']))"; }
run c3_sync --sync-obs && run c3_async && run c3_lazy --obs-lazy && run c4f_async --config c4f && \
run c5_sync --config c5 --steps 300 --warmup 30 --sync-obs && run c5_async --config c5 --steps 300 --warmup 30 && run c5_lazy --config c5 --steps 300 --warmup 30 --obs-lazy && \
run c2_async --config c2 && run c4_async --config c4
