#!/bin/bash
# Every BASELINE config as a bench line (no tests): c3 (default) c4 c4f c3-fear-off c2 c5 c1.
# Usage: tools/gpu_bench_all.sh TAG [steps]
TAG=${1:-all}; S=${2:-400}; O=gpurun_out/$TAG
mkdir -p $O; rm -f $O/*.log
run() { tag=$1; shift; timeout -k 10 240 python bench.py --steps $S --warmup 20 --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; python3 -c "
import json; l=[x for x in open('$O/$tag.log') if x.startswith('{')][-1]; j=json.loads(l); print('$tag', '%.4g' % j['value'], round(j['ms_per_step'],4), 'frac', round(j['roofline']['frac'] or 0,3), {k: (round(v,4) if isinstance(v,float) else v) for k,v in j['kernels_ms'].items() if k != 'kernel_path'})"; }
run c3 && run c4 --config c4 && run c4f --config c4f && run c3_f0 --fear 0 && run c2 --config c2 && run c5 --config c5 --steps 200 && run c5u --config c5 --steps 200 --updates-per-step 1
