"""Throughput of SURVEY §8f's "next" rows (the callers and formats either side of the hot path),
one JSON line each, for profiles/r2_next/.  Run on the GPU box:  python tools/bench_next.py

  f1  MADDPG update (maddpg/agent.py:199-224): batch 128, K = 2, 32x32; eager and one HIP-graph
      replay per update (sampling from a replay ring included in the graph)
  f2  evaluation (customeval.py:70-133): E episodes in parallel, eval-mode fused actor, cap 150
  f3  single-agent CustomEnv (custom/customenv.py:78-183): 65,536 envs of Level 3, FeAR on
  f4  Responsibility.FeAR + FeAL matrices (Responsibility.py:57-132, 213-303): snapshots per second
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-responsible-nav_amd")]

import torch  # noqa: E402


def timed(fn, n, sync=True):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    if sync:
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def f1():
    from marlnav.maddpg import MADDPG
    from marlnav.rollout import Rollout
    from marlnav.vec_env import VecGridEnv
    env = VecGridEnv("grid32", num_envs=4096, fear=True, fear_weight=-5.0, seed=1, stats=True, final_obs=True)
    m = MADDPG(env.K, env.H, env.W, device=env.device, seed=1, capturable=True)
    ro = Rollout(env, m.actors, replay_slots=16, training=True, seed=2)
    ro.reset()
    for _ in range(8):
        ro.step()
    ro.fence()
    for _ in range(5):  # kernel loading / GEMM selection outside the timing
        m.learn_from(ro.replay)
    eager = timed(lambda: m.learn_from(ro.replay), 30)
    m.capture(ro.replay)
    graph = timed(m.replay_learn, 200)
    env.close()
    return {"row": "f1 MADDPG learn", "batch": 128, "agents": 2, "obs": [32, 32], "ms_per_update_eager": eager * 1e3,
            "ms_per_update_graph": graph * 1e3, "updates_per_s": 1.0 / graph}


def f2():
    from marlnav.actor import MultiAgentActors
    from marlnav.evaluate import evaluate
    actors = MultiAgentActors(2, 32, 32, "mlp", device="cuda", seed=3)
    evaluate(actors, "grid32", episodes=1024, max_steps=150, fear=True)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = evaluate(actors, "grid32", episodes=65536, max_steps=150, fear=True)
    dt = time.perf_counter() - t0
    return {"row": "f2 evaluation", "episodes": 65536, "seconds": dt, "env_steps": out["steps"],
            "env_steps_per_s": out["steps"] / dt, "episodes_per_s": 65536 / dt,
            "crashes": out["crashes"], "apples_caught": out["apples_caught"]}


def f3():
    from marlnav.vec_env import VecGridEnv
    E = 65536
    env = VecGridEnv("level3_single", num_envs=E, fear=True, fear_weight=-5.0, variant="single", seed=4, stats=True)
    env.set_obs_async(True)
    env.reset()
    for _ in range(20):
        env.step()
    n = 300
    dt = timed(env.step, n)
    env.obs_fence()
    env.close()
    return {"row": "f3 single-agent CustomEnv", "envs": E, "us_per_step": dt * 1e6, "env_steps_per_s": E / dt,
            "kernel_path": env.kernel_path}


def f4():
    from marlnav import scenario as S
    from marlnav.vec_env import VecGridEnv
    out = []
    for name, n in (("grid32", 65536), ("grid64_n8", 16384)):
        sc = S.builtin(name)
        env = VecGridEnv(sc, num_envs=1, fear=True, seed=5)
        g = torch.Generator(device="cuda").manual_seed(6)
        road = torch.as_tensor(S.builtin(name).region.reshape(-1).nonzero()[0], device="cuda", dtype=torch.int32)
        idx = torch.stack([torch.randperm(road.numel(), device="cuda", generator=g)[: sc.N] for _ in range(64)])
        cells = road[idx].repeat(n // 64, 1).contiguous()
        acts = torch.randint(0, 9, (n, sc.N), device="cuda", generator=g, dtype=torch.int32)
        env.fear_matrix(cells[:64], acts[:64])
        dt = timed(lambda: env.fear_matrix(cells, acts), 5)
        out.append({"row": "f4 FeAR + FeAL matrices", "scenario": name, "agents": sc.N, "snapshots": n,
                    "ms_per_call": dt * 1e3, "snapshots_per_s": n / dt})
        env.close()
    return out


def main():
    which = sys.argv[1:] or ["f1", "f2", "f3", "f4"]
    for w in which:
        r = globals()[w]()
        for line in (r if isinstance(r, list) else [r]):
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
