#!/bin/bash
# Round 6: the whole GPU suite, then every config's bench line, then the C3 rocprofv3 evidence.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/tools/gpu_r6_lines.sh r6lines || exit 1
bash $R/tools/gpu_profile.sh r6_c3 --config c3 --steps 50 --warmup 10 || exit 1
