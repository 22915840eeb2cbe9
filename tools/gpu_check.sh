#!/bin/bash
# One GPU round trip: GPU test suite, per-phase cycle timing, benches (C3 default, C4f, C3 fear off, C2).
# Usage: tools/gpu_check.sh TAG [notests]
TAG=${1:-chk}; O=gpurun_out/$TAG
mkdir -p $O; rm -f $O/*.log
if [ "$2" != "notests" ]; then
  echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && exit 1
fi
echo "== phases" && timeout -k 10 300 python tools/phase_timing.py grid32 65536 > $O/phase.log 2>&1 && grep -A12 "step_v2<DEFER>" $O/phase.log || exit 1
B="python bench.py --steps 400 --warmup 20 --no-cpu-baseline"
run() { tag=$1; shift; env "$@" timeout -k 10 200 $B $EXTRA > $O/$tag.log 2>&1 || return 1; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', round(j['ms_per_step'],4), {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items() if k != 'kernel_path'})" || tail -3 $O/$tag.log; }
EXTRA="" && run c3 && EXTRA="--config c4f" && run c4f && EXTRA="--fear 0" && run c3_f0 && EXTRA="--config c2" && run c2
