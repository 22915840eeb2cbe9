"""Time the replay ring's batch-128 sample at C5's shape (65,536 envs, 32x32, K = 2): dense rows
(gw_replay_gather) vs rows expanded from the descriptor ring (gw_replay_gather_desc), GPU idle
otherwise.  Usage: python tools/bench_sample.py [E] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-responsible-nav_amd"))
from marlnav import scenario as S  # noqa: E402
from marlnav.actor import MultiAgentActors  # noqa: E402
from marlnav.rollout import Rollout  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=1, stats=True)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=0)
    ro = Rollout(env, actors, replay_slots=6, training=True, seed=2, obs_async=True, desc_ring=True)
    ro.reset()
    for _ in range(8):
        ro.step()
    ro.fence()
    rp = ro.replay
    g = torch.Generator(device="cuda").manual_seed(0)
    for use_desc in (False, True, False, True):
        for _ in range(10):
            rp._sample_hip(128, g, False, critic_in=True, use_desc=use_desc)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(iters):
            rp._sample_hip(128, g, False, critic_in=True, use_desc=use_desc)
        b.record()
        torch.cuda.synchronize()
        print(f"sample batch 128 ({'descriptor ring' if use_desc else 'dense rows'}): "
              f"{a.elapsed_time(b) / iters * 1000:.1f} us per call (incl. torch.rand / randint)", flush=True)
    env.close()


if __name__ == "__main__":
    main()
