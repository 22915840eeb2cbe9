#!/bin/bash
# Descriptor learner block stamps (GW_LEARN_STAMP): per-launch / per-block-type phase times.
T=${1:-r5s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O; rm -f $O/stamps.bin
MARLNAV_MEASURE=1 GW_LEARN_STAMP=$O/stamps.bin timeout -k 10 200 python tools/bench_desc_learn.py 65536 30 > $O/learn.log 2>&1 || { tail -5 $O/learn.log; exit 1; }
python tools/learn_stamps.py $O/stamps.bin 5 | tee $O/stamps.txt
