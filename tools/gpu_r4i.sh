# round 4 (i): window writer ablations at c5patch's shape: where its time goes
O=gpurun_out/r4i; mkdir -p $O
for v in "MODE=3" "MODE=3 PROBE=1" "MODE=3 PROBE=2" "MODE=9" "MODE=2" "MODE=2 PROBE=2"; do
  set -- $v; m=${1#MODE=}; pr=${2#PROBE=}
  if [ -n "$2" ]; then export GW_PATCH_PROBE=$pr; else unset GW_PATCH_PROBE; fi
  GW_PATCH_MODE=$m timeout -k 10 120 python tools/patch_probe.py 65536 11 > $O/p11_${m}_${pr}.log 2>&1 || exit 1
  GW_PATCH_MODE=$m timeout -k 10 120 python tools/patch_probe.py 65536 16 > $O/p16_${m}_${pr}.log 2>&1 || exit 1
  echo "$v: $(tail -1 $O/p11_${m}_${pr}.log) | $(tail -1 $O/p16_${m}_${pr}.log)"
done
