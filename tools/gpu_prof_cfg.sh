#!/bin/bash
# rocprofv3 kernel trace + stats of one bench config.  Usage: tools/gpu_prof_cfg.sh TAG CONFIG [bench args]
T=$1; CFG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; O=$ROOT/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $ROOT/bench.py --config $CFG --no-cpu-baseline "$@" > $O/prof.log 2>&1 || exit 1
python3 $ROOT/tools/bench_line.py $O/prof.log $CFG
f=$(find $O/prof -name '*kernel_stats.csv' | head -n 1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.1f} us {100*float(r["TotalDurationNs"])/tot:5.1f} %')
PY
