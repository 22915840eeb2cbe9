#!/bin/bash
# Round-5 profiles refreshed after the nontemporal row writer and the learner's LDS action rows.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_profile.sh r5_c4patch --config c4patch --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r5_c5patch --config c5patch --steps 50 --warmup 10 || exit 1
bash $R/tools/gpu_profile.sh r5_c5u1 --config c5 --updates-per-step 1 --steps 50 --warmup 10 || exit 1
