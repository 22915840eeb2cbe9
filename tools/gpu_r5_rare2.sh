#!/bin/bash
# Rare kernel with its input loads ahead of the weight staging: CNN-head tests, stamps, c4patch lines.
T=${1:-r5rare2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O; rm -f $O/rare.bin
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch_cnn.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 2 $O/pytest.log; [ $s = 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit $s; }
GW_RARE_STAMP=$O/rare.bin timeout -k 10 300 python bench.py --config c4patch --steps 30 --warmup 5 --graph 0 --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
python tools/rare_stamps.py $O/rare.bin 512 | head -1
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c4patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c4p_$i.log 2>&1 || exit 1
  python tools/bench_line.py $O/c4p_$i.log
done
