O=gpurun_out/learner; mkdir -p $O
timeout -k 10 120 python tools/bench_next.py f1 > $O/f1_fused.log 2>&1 && GW_LN_FUSED=0 timeout -k 10 120 python tools/bench_next.py f1 > $O/f1_torchln.log 2>&1
