mkdir -p gpurun_out/abl
B="python bench.py --steps 100 --warmup 10 --no-cpu-baseline"
for path in split fused; do for fear in 1 0; do
  echo "== $path fear=$fear" && GW_KERNEL=$path timeout -k 10 200 $B --fear $fear > gpurun_out/abl/${path}_f$fear.log 2>&1; python3 -c "
import json,sys; l=[x for x in open('gpurun_out/abl/${path}_f$fear.log') if x.startswith('{')][-1]; j=json.loads(l); print(j['ms_per_step'], j['kernels_ms'], j['roofline']['kernel'], round(j['roofline']['achieved']))"
done; done
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/abl
echo "== pmc sq split" && GW_KERNEL=split timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/sq_split -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/sq_split.log 2>&1 && echo ok
echo "== pmc sq fused" && GW_KERNEL=fused timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/sq_fused -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/sq_fused.log 2>&1 && echo ok
