# round 4 (l): the whole GPU suite + smoke, then the window writer / C3 / learner measurements
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -5 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 120 python tools/patch_probe.py > $O/probe_m4.log 2>&1 && tail -6 $O/probe_m4.log &&
timeout -k 10 120 python tools/patch_probe.py 65536 11 grid32 stamps > $O/probe_stamps_c5patch.log 2>&1 && tail -3 $O/probe_stamps_c5patch.log &&
timeout -k 10 300 python bench.py --config c5patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c5patch.log 2>&1 && python tools/bench_line.py $O/c5patch.log c5patch &&
timeout -k 10 300 python bench.py --config c4patch --steps 20 --warmup 5 --no-cpu-baseline > $O/c4patch.log 2>&1 && python tools/bench_line.py $O/c4patch.log c4patch &&
timeout -k 10 150 python tools/bench_learn.py 128 > $O/learn.log 2>&1 && tail -2 $O/learn.log &&
timeout -k 10 300 python bench.py > $O/c3_default.log 2>&1 && python tools/bench_line.py $O/c3_default.log c3_default
