#!/bin/bash
# A/B with arbitrary bench args: tools/gpu_ab2.sh TAG "bench args" "ENV=.." "ENV=.." ...
TAG=$1; shift; ARGS=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
i=0
for SET in "$@"; do
  i=$((i+1)); L=$O/run$i.log
  env $SET timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-cpu-baseline $ARGS > $L 2>&1 || { echo "FAILED: $SET"; tail -3 $L; exit 1; }
  python3 -c "
import json; l=[x for x in open('$L') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']
print('$ARGS'.ljust(22), '$SET'.ljust(30), round(j['ms_per_step'],4), 'step', round(k['step_kernel'],4), 'obs', round(k['obs_kernel'],4), 'fear', round(k['fear_kernel'],4))"
done
