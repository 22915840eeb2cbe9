#!/bin/bash
# Short-run bench A/B (the driver runs --steps 20 --warmup 5): pipeline events with / without
# the system-scope fence, profiling on / off, C2 graph / eager.  gpurun_out/short_ab/
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/short_ab; mkdir -p $O
run() { # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python - "$O/$n.log" "$n" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(f"{sys.argv[2]:>14}: {d['value']/1e9:.3f} G  {d['ms_per_step']*1e3:.1f} us/step  stream {k['stream_ms_per_step']*1e3:.1f}  "
      f"obs {k['obs_kernel']*1e3:.1f} step {k['step_kernel']*1e3:.1f} fear {k['fear_kernel']*1e3:.1f} (n={k['profiled_steps']}) "
      f"frac {d['roofline']['frac']}")
EOF
}
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1; s=$?; tail -n 3 $O/pytest_new.log; [ $s = 0 ] || exit $s
fi
for rep in 1 2; do
run d20_$rep --steps 20 --warmup 5 &&
run d20_p0_$rep --steps 20 --warmup 5 --profile-every 0 &&
GW_EVENT_FENCE=system run d20_sys_$rep --steps 20 --warmup 5 || exit 1
done
run s1000 --steps 1000 --warmup 100 &&
GW_EVENT_FENCE=system run s1000_sys --steps 1000 --warmup 100 &&
run c2 --config c2 &&
run c2_eager --config c2 --graph 0 &&
run c2_g64 --config c2 --graph 64 &&
run c5 --config c5 --steps 300 --warmup 30 &&
run bf16 --obs-dtype bf16 &&
run c4cnn --config c4cnn --steps 200 --warmup 20 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $O/prof.log 2>&1 && ls $O/prof
