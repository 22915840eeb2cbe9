# round 4 (t): the update replayed as a HIP graph vs issued eagerly inside C5 (one update per step)
O=gpurun_out/r4t; mkdir -p $O
for m in graph eager; do
  extra=""; [ $m = eager ] && extra="--eager-learn"
  timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline $extra > $O/c5u1_$m.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5u1_$m.log "c5u1 $m" | head -1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/eagerprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 --eager-learn > $GRAFT_REPO_ROOT/$O/eagerprof.log 2>&1) || exit 1
