#!/bin/bash
# fused CNN actor in isolation (tools/cnn_ab.py) + stream-priority A/B of the c4cnn / c5 / c3 benches
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/cnn2; mkdir -p $O
echo "== cnn_ab" && timeout -k 10 300 python tools/cnn_ab.py > $O/ab.log 2>&1 && cat $O/ab.log &&
for c in c4cnn c5 c3; do
  for pr in "" "--high-prio"; do
    echo "== $c $pr" && timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline $pr > $O/b_$c$pr.log 2>&1 && grep "^{" $O/b_$c$pr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels_ms'])" || exit 1
  done
done
