#!/bin/bash
# Round-5: the learner's tests + profile, then c4patch kernel stats for the window-writer / CNN-listing
# variants (default, GW_PATCH_PERSIST=0, GW_WCNN_LIST=scan).  Output: gpurun_out/$1/
T=${1:-r5c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_desc_learner.py tests/test_maddpg_fused.py -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -n 4 $O/pytest.log; [ $s = 0 ] || exit $s
bash $R/tools/gpu_r5_lprof.sh $T || exit 1
timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c5u1.log 2>&1 || exit 1
python tools/bench_line.py $O/bench_c5u1.log
cd /tmp && export TMPDIR=/tmp
for v in def persist0 scan; do
  case $v in def) e="";; persist0) e="GW_PATCH_PERSIST=0";; scan) e="GW_WCNN_LIST=scan";; esac
  if [ -n "$e" ]; then export ${e%%=*}=${e#*=}; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run --output-format csv -- python3 $R/bench.py --config c4patch --steps 200 --warmup 20 --no-cpu-baseline > $O/c4p_$v.log 2>&1 || exit 1
  unset GW_PATCH_PERSIST GW_WCNN_LIST
  f=$(find $O/p_$v -name '*kernel_stats.csv' | head -1) && cp $f $O/c4p_${v}_stats.csv && echo "== $v" && head -8 $O/c4p_${v}_stats.csv | cut -d, -f1-5 | cut -c1-160
done
