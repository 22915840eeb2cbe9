#!/bin/bash
# Window writer: its tests, c4patch / c5patch lines and the c4patch kernel stats.  Output: gpurun_out/$1/
T=${1:-r5win}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_obs_patch.py tests/test_gpu_patch_cnn.py -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 3 $O/pytest.log; [ $s = 0 ] || exit $s
for c in c4patch c5patch; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit 1
  python tools/bench_line.py $O/bench_$c.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --config c4patch --steps 100 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name '*kernel_stats.csv' | head -1) && cp $f $O/c4patch_kernel_stats.csv && head -9 $O/c4patch_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
