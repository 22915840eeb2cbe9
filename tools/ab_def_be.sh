#!/bin/bash
# A/B: the deferred-FeAR world update on 32-env blocks with lane-parallel draws (-DGW_DEF_BE=32, csrc/build_ab/wt_def32) vs 128-env blocks (release); C5 and C3
O=gpurun_out/ab_defbe; mkdir -p $O
L=$PWD/marl-responsible-nav_amd/csrc/build_ab/wt_def32/libgridenv.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/c5_rel_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c5_rel_$i.log | sed "s/^/rel /" | tee -a $O/summary.txt
  MARLNAV_LIB=$L timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline > $O/c5_def32_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c5_def32_$i.log | sed "s/^/def32 /" | tee -a $O/summary.txt
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_rel_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c3_rel_$i.log | sed "s/^/rel /" | tee -a $O/summary.txt
  MARLNAV_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_def32_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c3_def32_$i.log | sed "s/^/def32 /" | tee -a $O/summary.txt
done
