#!/bin/bash
# Round 6 end: rocprofv3 evidence (trace + FETCH / WRITE / VALU passes) of every rollout / window config on the final build
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r6_c5 --config c5 --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r6_c2 --config c2 --steps 200 --warmup 20 || exit 1
bash $R/tools/gpu_profile.sh r6_c5u1 --config c5 --updates-per-step 1 --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r6_c5patch --config c5patch --steps 100 --warmup 20 || exit 1
bash $R/tools/gpu_profile.sh r6_c4patch --config c4patch --steps 100 --warmup 20 || exit 1
bash $R/tools/gpu_profile.sh r6_c4f --config c4f --steps 20 --warmup 5 || exit 1
