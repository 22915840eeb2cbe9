"""A/B timing of the fused CNN actor (gw_cnn_act = cnn_l1_kernel + act_kernel<H1>) in isolation,
with phases switched off through GW_CNN_AB (bit 0: the recomputed positions, bit 1: the table
rows).  Eager launches timed with events around `iters` calls on an otherwise idle GPU.
Run on the GPU box:  python tools/cnn_ab.py [scenario] [envs] [iters]"""
import os

# the A/B and probe switches exist only in the measurement build (csrc/measure.h)
os.environ.setdefault("MARLNAV_MEASURE", "1")
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-responsible-nav_amd")]

import torch  # noqa: E402

from marlnav.actor import MultiAgentActors  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    scen = sys.argv[1] if len(sys.argv) > 1 else "grid64_n8"
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    env = VecGridEnv(scen, num_envs=E, fear=False, seed=1)
    actors = MultiAgentActors(env.K, env.H, env.W, "cnn", device=env.device, seed=2)
    env.reset()
    for _ in range(8):
        env.step()
    mask = env.out["mask"]
    a = torch.empty((E, env.K), dtype=torch.int32, device="cuda")
    pr = torch.empty((env.K, E, 9), dtype=torch.float32, device="cuda")
    actors.act_env(env, mask, True, seed=1, counter=0, actions_out=a, probs_out=pr)  # prepare
    torch.cuda.synchronize()
    t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t[0].record()
    actors.mark_updated()
    actors.act_env(env, mask, True, seed=1, counter=0, actions_out=a, probs_out=pr)  # prepare + act
    t[1].record()
    torch.cuda.synchronize()
    print(f"prepare + act: {t[0].elapsed_time(t[1]) * 1e3:.1f} us", flush=True)
    for ab in [0, 1, 2, 3]:
        os.environ["GW_CNN_AB"] = str(ab)
        for _ in range(5):
            actors.act_env(env, mask, True, seed=1, counter=0, actions_out=a, probs_out=pr)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for i in range(iters):
            actors.act_env(env, mask, True, seed=1, counter=i, actions_out=a, probs_out=pr)
        e1.record()
        torch.cuda.synchronize()
        print(f"GW_CNN_AB={ab}: {e0.elapsed_time(e1) / iters * 1e3:.1f} us per gw_cnn_act", flush=True)
    os.environ["GW_CNN_AB"] = "0"
    env.close()


if __name__ == "__main__":
    main()
