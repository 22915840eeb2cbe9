#!/bin/bash
# HBM read/write ceilings + a rocprofv3 kernel trace of the full-rollout (c5) bench
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c5prof; mkdir -p $O
[ "$1" = "probe" ] && { echo "== probe" && timeout -k 10 120 ./tools/hbm_probe2 537 > $O/probe.log 2>&1 && cat $O/probe.log; }
cd /tmp && export TMPDIR=/tmp &&
echo "== c5 trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline --profile-every 0 $EXTRA > $O/c5.log 2>&1 && tail -1 $O/c5.log | cut -c1-300 &&
python3 -c "
import csv,glob
f=glob.glob('$O/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:30]: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['Percentage']),1), r['Name'][:150])"
