#!/bin/bash
# The whole GPU suite (as the driver runs it), one process.  Output: gpurun_out/$1/
T=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; s=$?
grep -E "passed|failed|error" $O/pytest.log | tail -3; exit $s
