# round 4 (y): the critic tail on three 4-wave groups (critic_tail3) vs one (GW_TAIL_PAR=0)
O=gpurun_out/r4y; mkdir -p $O
for v in 0 4 8; do
  GW_TAIL_PAR=$v timeout -k 10 120 python tools/tail_ab.py $O/w_$v.safetensors > $O/tail_ab_$v.log 2>&1 || exit 1
done
python - <<'PY' || exit 1
from safetensors.torch import load_file
import torch
a = load_file("gpurun_out/r4y/w_0.safetensors")
for v in ("4", "8"):
    b = load_file(f"gpurun_out/r4y/w_{v}.safetensors")
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    print("GW_TAIL_PAR", v, "bit-identical to the one-group tail:", not bad, bad[:3])
    assert not bad
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_maddpg_fused.py tests/test_maddpg.py tests/test_gpu_replay_desc.py > $O/pytest.log 2>&1; s=$?; tail -2 $O/pytest.log; [ $s = 0 ] || exit $s
for v in 0 4 8; do
  GW_TAIL_PAR=$v timeout -k 10 120 python tools/bench_learn.py 128 > $O/learn_$v.log 2>&1 || exit 1
  echo "GW_TAIL_PAR=$v: $(tail -2 $O/learn_$v.log | tr '\n' ' ')"
  GW_TAIL_PAR=$v timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 200 --warmup 10 --no-cpu-baseline > $O/c5u1_$v.log 2>&1 || exit 1
  python tools/bench_line.py $O/c5u1_$v.log "c5u1 GW_TAIL_PAR=$v" | head -1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --updates-per-step 1 --steps 50 --warmup 10 --no-cpu-baseline --profile-steps 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || exit 1
