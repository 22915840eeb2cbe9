"""Fused CNN get_action (gw_cnn_act, include/actor_ops.h) against the PyTorch fp32 CNN head
(nn.Conv2d -> ReLU -> nn.Conv2d -> ReLU -> flatten -> Linear ... ; configs/cnn.yaml:2-6,
maddpg/agent.py:94-100) on the dense observations the env wrote.

The kernel never reads the observation: layer 1 = z_map + the changed conv-2 positions' deltas,
from a per-(agent, position, cell, value) table or, where one position holds several patched
cells, by recomputing that position.  It differs from torch's dense path only in f32 summation
order (a 16,384-long Linear-1 dot as z_map + deltas).  Tolerances (stated here): logits
|d| <= 5e-4 + 5e-4 |x|; probs |d| <= 5e-5; actions equal wherever the best masked probability
leads the runner-up by more than 1e-3.  Gumbel uniforms are passed in so both paths see the
same noise.
"""
import numpy as np
import pytest
import torch

from marlnav import scenario as S
from marlnav.actor import MultiAgentActors, N_ACTIONS
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _dense_logits(actors, obs):
    """torch fp32 reference: the nn.Conv2d form (not the per-patch GEMM form) of every agent."""
    out = []
    for k, n in enumerate(actors.nets):
        x = obs[k].float().unsqueeze(1)
        out.append(n.mlp(n.conv(x).flatten(1)))
    return torch.stack(out)


def _multi_patch_fraction(env, sc):
    """Share of (env, agent) pairs whose observation has a conv-2 position holding 2+ patched cells."""
    pos = env.positions().cpu().numpy()          # [E, N]
    E = pos.shape[0]
    hits = 0
    for k in range(sc.K):
        cells = np.concatenate([pos, np.full((E, 1), sc.apples[k])], 1)
        reg = (cells // sc.W // 4) * (sc.W // 4) + (cells % sc.W) // 4
        srt = np.sort(reg, 1)
        hits += int((srt[:, 1:] == srt[:, :-1]).any(1).sum())
    return hits / (E * sc.K)


def _check(actors, env, training, seed):
    E, K = env.E, env.K
    mask = env.out["mask"]
    g = torch.Generator(device="cuda").manual_seed(seed)
    u = torch.rand((K, E, N_ACTIONS), device="cuda", generator=g)
    logits_k = torch.full((K, E, N_ACTIONS), float("nan"), device="cuda")
    a_k, p_k = actors.act_env(env, mask, training, uniform=u, logits_out=logits_k)
    with torch.no_grad():
        logits_r = _dense_logits(actors, env.out["obs"])
    z = logits_r - torch.log(-torch.log(u + 1e-20) + 1e-20) if training else logits_r
    probs_r = torch.softmax(z, dim=-1)
    bits = (mask.t().to(torch.int32).unsqueeze(-1) >> torch.arange(N_ACTIONS, device=mask.device)) & 1
    pm_r = torch.where(bits.bool(), probs_r, torch.zeros((), device=probs_r.device))
    torch.testing.assert_close(logits_k, logits_r, rtol=5e-4, atol=5e-4)
    torch.testing.assert_close(p_k, probs_r, rtol=0, atol=5e-5)
    top2 = pm_r.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1] > 1e-3).t()
    want = pm_r.argmax(-1).t().to(torch.int32)
    assert bool(clear.float().mean() > 0.5)
    assert torch.equal(a_k[clear], want[clear])
    assert bool(((mask.long() >> a_k.long()) & 1).all())
    return a_k


@pytest.mark.parametrize("scen,E,fear,steps", [("grid64_n8", 65536, False, 6), ("grid64_n8", 3000, True, 25),
                                               ("grid32", 4096, True, 25)])
def test_fused_cnn_act_matches_torch_conv(scen, E, fear, steps):
    sc = S.builtin(scen)
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=5, max_steps=12)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "cnn", device="cuda", seed=3)
    assert actors.fusable(env)
    env.reset()
    _check(actors, env, training=True, seed=0)          # reset encoding (0.5 agents, 9.5 / 9 apples)
    multi = []
    for t in range(steps):                              # step encoding, relabels, auto-resets (12-step cap)
        a = actors.act_env(env, env.out["mask"], training=(t % 2 == 0), seed=1, counter=t)[0]
        env.step(a)
        multi.append(_multi_patch_fraction(env, sc))
        if t % 3 == 0 or t == steps - 1:
            _check(actors, env, training=(t % 2 == 1), seed=t + 1)
    assert max(multi) > 0.01, "no position with several patched cells was exercised"
    env.close()


def test_fused_cnn_follows_weight_updates_and_rejects_unfusable():
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=512, fear=False, seed=2)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "cnn", device="cuda", seed=8)
    env.reset()
    env.step()
    _check(actors, env, training=False, seed=1)
    with torch.no_grad():  # an in-place parameter change must re-derive the tables
        for n in actors.nets:
            n.conv[2].weight.mul_(-1.5)
            n.mlp[0].bias.add_(0.3)
    _check(actors, env, training=False, seed=2)
    env.close()
    lv = S.builtin("level3")  # 10 x 16: H not a multiple of 4
    env3 = VecGridEnv(lv, num_envs=4, fear=False, seed=2)
    a3 = MultiAgentActors(lv.K, lv.H, lv.W, "cnn", device="cuda", seed=1)
    assert not a3.fusable(env3)
    env3.close()
