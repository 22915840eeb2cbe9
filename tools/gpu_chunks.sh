#!/bin/bash
# obs-writer chunking (GW_OBS_CHUNKS) A/B on c4cnn / c5 / c3, lazy and eager, + c4cnn timeline
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/chunks; mkdir -p $O
for c in c4cnn c5 c3; do
  for ch in 1 4 8 16; do
    for m in "" "--obs-eager"; do
      [ "$c" = c3 ] && [ -n "$m" ] && continue
      echo -n "== $c chunks=$ch $m: " && GW_OBS_CHUNKS=$ch timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline $m > $O/b_${c}_${ch}$m.log 2>&1 && grep "^{" $O/b_${c}_${ch}$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" || exit 1
    done
  done
done
cd /tmp && export TMPDIR=/tmp &&
echo "== trace c4cnn chunks 8" && GW_OBS_CHUNKS=8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4cnn --steps 30 --warmup 5 --no-cpu-baseline --profile-every 0 > $O/t.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/timeline.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) step_v2 1
