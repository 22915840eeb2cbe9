# round 4: the whole GPU suite + smoke, as the driver runs them at round end
O=gpurun_out/r4_full; mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?; tail -5 $O/pytest.log; [ $s = 0 ] || exit $s
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; s=$?; tail -3 $O/smoke.log; exit $s
