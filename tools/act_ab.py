"""A/B timing of the fused actor kernel (gw_actor_act) with phases switched off through GW_ACT_AB
(bit 0: W1 gathers, bit 1: layer-2 MFMAs, bit 2: epilogue) and, with bit 3, per-phase s_memtime
stamps of wave 0 of every block.  Run on the GPU box:
    python tools/act_ab.py [scenario] [envs] [iters]"""
import ctypes as C
import os

# the A/B and probe switches exist only in the measurement build (csrc/measure.h)
os.environ.setdefault("MARLNAV_MEASURE", "1")
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-responsible-nav_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlnav import _lib  # noqa: E402
from marlnav.actor import MultiAgentActors  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    scen = sys.argv[1] if len(sys.argv) > 1 else "grid32"
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    env = VecGridEnv(scen, num_envs=E, fear=True, seed=1)
    actors = MultiAgentActors(env.K, env.H, env.W, "mlp", device=env.device, seed=2)
    env.reset()
    for _ in range(5):
        env.step()
    mask = env.out["mask"]
    a = torch.empty((E, env.K), dtype=torch.int32, device="cuda")
    pr = torch.empty((env.K, E, 9), dtype=torch.float32, device="cuda")
    for ab in [int(x) for x in os.environ.get("ACT_AB_LIST", "0,1,2,4,3,7,6,5,16,23").split(",")]:
        os.environ["GW_ACT_AB"] = str(ab)
        actors.act_env(env, mask, True, seed=1, counter=0, actions_out=a, probs_out=pr)  # prepare outside
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()  # one launch captured: replays time the kernel, not the host
        with torch.cuda.graph(g):
            actors.act_env(env, mask, True, seed=1, counter=0, actions_out=a, probs_out=pr)
        for _ in range(10):
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for i in range(iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"GW_ACT_AB={ab}: {e0.elapsed_time(e1) / iters * 1e3:.1f} us per launch (graph replay)", flush=True)
    t0 = __import__("time").perf_counter()
    os.environ["GW_ACT_AB"] = "0"
    for i in range(iters):
        actors.act_env(env, mask, True, seed=1, counter=i, actions_out=a, probs_out=pr)
    torch.cuda.synchronize()
    print(f"eager act_env: {(__import__('time').perf_counter() - t0) / iters * 1e6:.1f} us per call", flush=True)
    os.environ["GW_ACT_AB"] = "8"
    actors.act_env(env, mask, True, seed=1, counter=0, actions_out=a, probs_out=pr)
    torch.cuda.synchronize()
    buf = np.zeros((1024, 16), np.uint64)
    lib = _lib.load()
    lib.gw_actor_debug_clocks.argtypes = [C.c_void_p, C.c_int]
    assert lib.gw_actor_debug_clocks(buf.ctypes.data, 1024) == 0
    nb = min(1024, 512)
    t = buf[:nb].astype(np.int64)
    t0 = t[:, 0].min()
    names = ["start", "staged", "t0 desc", "t0 layer1", "t0 ln1", "t0 mfma", "t0 end", "t1 desc", "t1 layer1",
             "t1 ln1", "t1 mfma", "t1 end"]
    print("phase (block wave 0, cycles since the first block's start): mean / p10 / p90")
    for i, nm in enumerate(names):
        col = t[:, i]
        ok = col > 0
        if not ok.any():
            continue
        v = col[ok] - t0
        print(f"  {nm:10s} {v.mean():9.0f} {np.percentile(v, 10):9.0f} {np.percentile(v, 90):9.0f}")
    env.close()


if __name__ == "__main__":
    main()
