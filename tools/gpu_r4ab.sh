# round 4 (ab): the descriptor gather with both agents of a row in one 512-thread block (GW_GATHER_KB=2)
O=gpurun_out/r4ab; mkdir -p $O
GW_GATHER_KB=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay_desc.py > $O/pytest_kb2.log 2>&1; s=$?; tail -2 $O/pytest_kb2.log; [ $s = 0 ] || exit $s
for kb in 1 2; do
  GW_GATHER_KB=$kb timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline > $O/c5u1_kb$kb.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5u1_kb$kb.log "c5u1 GW_GATHER_KB=$kb" | head -1
done
(cd /tmp && export TMPDIR=/tmp && GW_GATHER_KB=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || exit 1
