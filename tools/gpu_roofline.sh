#!/bin/bash
# Per-config roofline evidence: for each CONFIG, the driver-size bench line (live spans of every
# kernel kind), then rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes of the
# same command (tools/gpu_profile.sh).  Usage: tools/gpu_roofline.sh TAG CONFIG...  -> gpurun_out/TAG/
T=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$T; mkdir -p $O
for C in "$@"; do
  echo "== $C"
  timeout -k 10 300 python $ROOT/bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -5 $O/bench_$C.log; exit 1; }
  python $ROOT/tools/bench_line.py $O/bench_$C.log $C
  bash $ROOT/tools/gpu_profile.sh ${T}_$C --config $C --steps 20 --warmup 5 > $O/profile_$C.log 2>&1 || { echo "profile $C failed"; tail -5 $O/profile_$C.log; exit 1; }
done
echo "== all done"
