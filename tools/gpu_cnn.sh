#!/bin/bash
# Fused CNN head (gw_cnn_act): parity tests, then the c4cnn rollout bench (fused vs PyTorch) and a
# rocprofv3 kernel trace of the fused one.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/cnn; mkdir -p $O
echo "== cnn tests" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn_actor.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || { grep -E "^E " $O/pytest.log | head -20; exit $s; }
echo "== bench c4cnn fused" && timeout -k 10 300 python bench.py --config c4cnn --steps 100 --warmup 10 --no-cpu-baseline > $O/bench.log 2>&1 && grep "^{" $O/bench.log | cut -c1-400 &&
echo "== bench c4cnn torch" && timeout -k 10 300 python bench.py --config c4cnn --steps 10 --warmup 2 --no-cpu-baseline --cnn-torch > $O/bench_torch.log 2>&1 && grep "^{" $O/bench_torch.log | cut -c1-300 &&
cd /tmp && export TMPDIR=/tmp &&
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4cnn --steps 50 --warmup 5 --no-cpu-baseline --profile-every 0 > $O/trace.log 2>&1 &&
python3 -c "
import csv,glob
f=glob.glob('$O/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['Percentage']),1), r['Name'][:110])"
