#!/bin/bash
# SQ (shader sequencer) counters per kernel, one rocprofv3 --pmc pass per counter group.
# Usage: tools/gpu_sq.sh TAG [bench args]   (kernels run serially: GW_DEFER=0)
TAG=${1:-sq}; shift
ARGS=${@:---steps 20 --warmup 5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && export GW_DEFER=${GW_DEFER:-0}
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  echo "== pass $i" && timeout -k 10 300 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 $ROOT/bench.py $ARGS --no-cpu-baseline --profile-every 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; break; }
done
python3 $ROOT/tools/sq_summary.py $OUT | tee $OUT/summary.txt
