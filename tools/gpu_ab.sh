#!/bin/bash
# A/B benches: tools/gpu_ab.sh TAG "ENV=.. ENV=.." "ENV=.." ...  (each arg = one env setting; C3 + C4f each)
TAG=$1; shift; O=gpurun_out/$TAG; mkdir -p $O
B="python bench.py --steps 400 --warmup 20 --no-cpu-baseline"
i=0
for SET in "$@"; do
  for CFG in c3 c4f; do
    i=$((i+1)); L=$O/run$i.log
    env $SET timeout -k 10 200 $B --config $CFG > $L 2>&1 || { echo "FAILED: $SET $CFG"; tail -3 $L; exit 1; }
    python3 -c "
import json; l=[x for x in open('$L') if x.startswith('{')][-1]; j=json.loads(l); k=j['kernels_ms']
print('$CFG', '$SET'.ljust(40), round(j['ms_per_step'],4), 'step', round(k['step_kernel'],4), 'obs', round(k['obs_kernel'],4), 'fear', round(k['fear_kernel'],4))"
  done
done
