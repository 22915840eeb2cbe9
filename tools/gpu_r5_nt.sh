#!/bin/bash
# Row writer A/B: nontemporal float4 stores (plain before: GW_PATCH_PROBE=8 was the A/B switch), alone, both patch shapes.
T=${1:-r5nt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
for pr in 0 0; do
  for sh in "65536 11 grid32" "65536 16 grid64_n8"; do
    MARLNAV_MEASURE=1 GW_PATCH_PROBE=$pr timeout -k 10 120 python tools/patch_probe.py $sh > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
    echo "probe=$pr $(grep GB/s $O/p.log)"
  done
done
