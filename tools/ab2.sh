#!/bin/bash
# same-box A/B: the working tree's library (new) vs csrc/build_ab/base (old), alternating.  Usage: tools/ab2.sh TAG "bench args" [reps]
T=$1; A=$2; N=${3:-2}
O=gpurun_out/ab_$T; mkdir -p $O
for i in $(seq $N); do
  MARLNAV_LIB=$PWD/marl-responsible-nav_amd/csrc/build_ab/base/libgridenv.so timeout -k 10 300 python bench.py $A --no-cpu-baseline > $O/old_$i.log 2>&1 || exit 1
  python tools/summ.py $O/old_$i.log | sed 's/^/old /' | tee -a $O/summary.txt
  timeout -k 10 300 python bench.py $A --no-cpu-baseline > $O/new_$i.log 2>&1 || exit 1
  python tools/summ.py $O/new_$i.log | sed 's/^/new /' | tee -a $O/summary.txt
done
