#!/bin/bash
# c4cnn pipeline A/B: lazy (default) / eager / synchronous obs writes, with kernel timelines
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/c4ab; mkdir -p $O
for m in "" "--obs-eager" "--sync-obs"; do
  echo "== c4cnn $m" && timeout -k 10 300 python bench.py --config c4cnn --steps 100 --warmup 10 --no-cpu-baseline $m > $O/b$m.log 2>&1 && grep "^{" $O/b$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" || exit 1
done
cd /tmp && export TMPDIR=/tmp &&
echo "== trace eager" && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_eager -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4cnn --steps 30 --warmup 5 --no-cpu-baseline --profile-every 0 --obs-eager > $O/te.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/timeline.py $(ls $O/trace_eager/*/run_kernel_trace.csv $O/trace_eager/run_kernel_trace.csv 2>/dev/null | head -1) step_v2 2
