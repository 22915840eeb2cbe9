#!/bin/bash
# Round-5 rocprofv3 evidence: trace + FETCH / WRITE / VALU passes per config (tools/gpu_profile.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r5_c3 --config c3 --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r5_c5u1 --config c5 --updates-per-step 1 --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r5_c4patch --config c4patch --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r5_c5patch --config c5patch --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r5_c4f --config c4f --steps 30 --warmup 5 || exit 1
