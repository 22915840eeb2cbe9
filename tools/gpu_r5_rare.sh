#!/bin/bash
# Rare-kernel block stamps at c4patch (GW_RARE_STAMP; eager steps).
T=${1:-r5rare}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O; rm -f $O/rare.bin
MARLNAV_MEASURE=1 GW_RARE_STAMP=$O/rare.bin timeout -k 10 300 python bench.py --config c4patch --steps 30 --warmup 5 --graph 0 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
python tools/rare_stamps.py $O/rare.bin 512 | tee $O/stamps.txt
