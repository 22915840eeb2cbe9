"""Measurement only: 300 C2-shape env steps (grid32, 4,096 envs, FeAR off): 0 without obs, 1 with
async obs (the merged step_obs kernel), 2 with synchronous obs (step_v2 + obs_kernel launches),
for rocprofv3 --kernel-trace --stats."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))
import torch
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv
mode = sys.argv[1]
env = VecGridEnv(S.builtin("grid32"), num_envs=4096, fear=False, seed=3, obs=mode != "0")
if mode == "1":
    env.set_obs_async(True)
env.reset()
for _ in range(300):
    env.step()
torch.cuda.synchronize()
print(env.kernel_path)
