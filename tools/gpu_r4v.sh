# round 4 (v): C5 with one update per step (recorded launches): obs streams confined to fewer CUs
O=gpurun_out/r4v; mkdir -p $O
for cus in 0 224 192 160 128; do
  export GW_OBS_CUS=$cus
  timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline --learn-launches > $O/c5u1_cus$cus.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5u1_cus$cus.log "c5u1 launches obs_cus=$cus" | head -1
done
export GW_OBS_CUS=0 GW_OBS_PRIO=lo
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline --learn-launches > $O/c5u1_lo.log 2>&1 || exit 1
python tools/bench_line.py $O/c5u1_lo.log "c5u1 launches obs prio lo" | head -1
unset GW_OBS_PRIO
export GW_OBS_CUS=192
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/cus192prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 --learn-launches > $GRAFT_REPO_ROOT/$O/cus192prof.log 2>&1) || exit 1
