"""Host enqueue cost of VecGridEnv.step vs the GPU time per step (is a config host bound?).
Run on the GPU box:  python tools/host_cost.py [scenario] [envs] [fear]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-responsible-nav_amd")]

import torch  # noqa: E402

from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    scen = sys.argv[1] if len(sys.argv) > 1 else "grid32"
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    fear = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
    for mode in (False, True):
        env = VecGridEnv(scen, num_envs=E, fear=fear, seed=1, stats=True)
        env.set_obs_async(mode)
        env.reset()
        for _ in range(50):
            env.step()
        torch.cuda.synchronize()
        n = 1000
        t0 = time.perf_counter()
        for _ in range(n):
            env.step()
        t1 = time.perf_counter()
        env.obs_fence()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{scen} E={E} fear={fear} async={mode}: host enqueue {(t1 - t0) / n * 1e6:.1f} us/step, "
              f"wall {(t2 - t0) / n * 1e6:.1f} us/step", flush=True)
        env.close()


if __name__ == "__main__":
    main()
