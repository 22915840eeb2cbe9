#!/bin/bash
# actor-op GPU tests, A/B phase timing and the c5 trace
mkdir -p gpurun_out/act
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_actor_ops.py tests/test_gpu_rollout.py > gpurun_out/act/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/act/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/act_ab.py grid32 65536 200 && bash tools/gpu_c5prof.sh && grep '^{' gpurun_out/c5prof/c5.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('c5 ms/step', j['ms_per_step'])"
