"""Measurement only: eager learn_desc vs recorded launches with the fused actor images, step by step."""
import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "marl-responsible-nav_amd"))
import torch
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv
from marlnav.maddpg import MADDPG
from marlnav.rollout import Rollout
sc = S.builtin("grid32")
runs = {}
for mode in ("eager", "launches"):
    env = VecGridEnv(sc, num_envs=512, fear=True, fear_weight=-5.0, stats=True, seed=7, max_steps=10)
    m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
    ro = Rollout(env, m.actors, replay_slots=16, training=True, seed=4, obs_async=True, desc_ring=True)
    ro.reset()
    log = []
    for t in range(8):
        ro.step()
        torch.cuda.synchronize()
        log.append(("probs", t, ro.replay.probs.clone()))
        if t < 2:
            continue
        ro.learn_fence()
        if mode == "eager":
            m.learn_desc(ro.replay)
        else:
            if m._graph is None:
                m.capture(ro.replay, actor_env=env, launches=True, warmup=1)
            else:
                m.replay_learn()
        torch.cuda.synchronize()
        log.append(("actor", t, m.actors.net.flat_params().clone()))
        log.append(("ws", t, m.actors._fast["ws"].clone()))
    runs[mode] = log
    env.close()
for (n, t, a), (_, _, b) in zip(runs["eager"], runs["launches"]):
    if n == "ws":
        K, HID = sc.K, 128
        a, b = a[K * HID:], b[K * HID:]
    eq = torch.equal(a.view(torch.int32), b.view(torch.int32))
    print(n, t, eq, "" if eq else int((a.view(torch.int32) != b.view(torch.int32)).sum()))
