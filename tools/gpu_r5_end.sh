#!/bin/bash
# Round-5 end check after the fused write-and-list: the whole suite, smoke, the driver's command,
# then rocprofv3 evidence for c4patch.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_final.sh r5final2 || exit 1
bash $R/tools/gpu_profile.sh r5_c4patch --config c4patch --steps 50 --warmup 10 > $R/gpurun_out/r5final2/prof_c4patch.log 2>&1; echo "c4patch profile rc $?"
