"""Measurement only: gw_patch_cnn_act at bench.py --config c4patch's size (or with "full":
gw_cnn_act at c4cnn's), CALLS act calls on a fixed env state (run under rocprofv3 --kernel-trace
--stats; GW_CNN_AB selects the A/B variants of the layer-1 kernels, csrc/actor_ops.hip).
Usage: wcnn_probe.py [CALLS] [full]"""
import os

# the A/B and probe switches exist only in the measurement build (csrc/measure.h)
os.environ.setdefault("MARLNAV_MEASURE", "1")
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))

import torch  # noqa: E402

from marlnav import scenario as S  # noqa: E402
from marlnav.actor import MultiAgentActors  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    full = "full" in sys.argv[2:]
    sc = S.builtin("grid64_n8")
    P = 0 if full else 16
    env = VecGridEnv(sc, num_envs=65536, fear=False, seed=8, max_steps=30, obs=full)
    actors = MultiAgentActors(sc.K, P or env.H, P or env.W, arch="cnn", device="cuda", seed=0)
    env.reset()
    for _ in range(5):
        env.step()
    for _ in range(calls):
        actors.act_env(env, env.out["mask"], True, seed=1, counter=0, patch=P)
    torch.cuda.synchronize()
    if full:
        env.close()
        return
    ws = actors._fast["ws"]
    rn = None
    try:  # items per (env, agent): rare_n sits right after rare_z in the workspace (wcnn_ws_layout)
        lib = actors._fast["lib"]
        n = int(lib.gw_patch_cnn_workspace_floats(P, env.H, env.W, sc.K, env.E))
        nblk = (env.E + 255) // 256  # rare_n, bucket_n, bucket, unit_off, qmask, cnt, off
        tail = sc.K * env.E + sc.K * 16 * (env.E + 2) + 1 + sc.K * env.E + 2 * sc.K * 16 * nblk
        rn = ws[n - tail:n - tail + sc.K * env.E].view(torch.int32)
        print("items per (env, agent): mean %.3f max %d" % (rn.float().mean().item(), rn.max().item()))
    except Exception as ex:  # noqa: BLE001
        print("rare_n unavailable:", ex)
    env.close()


if __name__ == "__main__":
    main()
