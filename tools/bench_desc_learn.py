"""Time the descriptor learner (gw_maddpg_desc_update) on a filled descriptor ring (C5 shapes:
32x32, K = 2, batch 128): eager calls and recorded launches, each alone on the GPU.
  python tools/bench_desc_learn.py [envs] [updates]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))
import torch  # noqa: E402

from marlnav import scenario as S  # noqa: E402
from marlnav.maddpg import MADDPG  # noqa: E402
from marlnav.rollout import Rollout  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, stats=True, seed=7, max_steps=150)
    m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
    ro = Rollout(env, m.actors, replay_slots=8, training=True, seed=4, obs_async=True, desc_ring=True)
    ro.reset()
    for _ in range(6):
        ro.step()
    ro.fence()
    rp = ro.replay
    assert m.desc_capable(rp)
    for _ in range(5):
        m.learn_desc(rp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        m.learn_desc(rp)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / n * 1e3
    m.capture(rp, launches=True, warmup=1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        m.replay_learn()
    e1.record()
    torch.cuda.synchronize()
    print(f"descriptor learner, batch {m.batch_size}, {E} envs: eager {eager:.3f} ms/update, "
          f"recorded launches {e0.elapsed_time(e1) / n:.3f} ms/update (GPU)", flush=True)
    env.close()


if __name__ == "__main__":
    main()
