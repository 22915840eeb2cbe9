#!/bin/bash
# A/B: c5u1 with the whole step chain (actor, env, MADDPG update) on a high-priority stream (--high-prio)
O=gpurun_out/ab_c5u1prio; mkdir -p $O
for i in 1 2; do for a in "" "--high-prio"; do
  n=$([ -z "$a" ] && echo main || echo prio)
  timeout -k 10 300 python bench.py --config c5 --updates-per-step 1 $a --steps 100 --warmup 20 --no-cpu-baseline > $O/c5u1_${n}_$i.log 2>&1 || exit 1
  python tools/summ.py $O/c5u1_${n}_$i.log | sed "s/^/$n /" | tee -a $O/summary.txt
done; done
