"""Fused get_action over each RL agent's P x P egocentric window (gw_patch_actor_act; X1, not a
reference format) against the PyTorch fp32 actor on the windows ``VecGridEnv.obs_patch(P)``
writes (themselves == -1-padded crops of the oracle-pinned full obs, tests/test_gpu_obs_patch.py).

Layer 1 starts from a per-centre-cell table (bias + the map window's W1 product, summed in
another order than torch's GEMM) plus one W1 row per patched cell inside the window; layers 2-3
are the full-grid actor's MFMA chain.  Tolerances as tests/test_actor_ops.py (f32 summation
order only): logits |d| <= 2e-4 + 2e-4 |x|; probs |d| <= 2e-5; actions equal wherever the best
masked probability leads the runner-up by more than 1e-4.
"""
import pytest
import torch

from marlnav import scenario as S
from marlnav.actor import MultiAgentActors, N_ACTIONS
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _actors(K, P, seed):
    actors = MultiAgentActors(K, P, P, "mlp", device="cuda", seed=seed)
    net = actors.net
    g = torch.Generator(device="cpu").manual_seed(seed + 100)
    with torch.no_grad():  # non-trivial LayerNorm affine and biases
        for i in range(2):
            net.ln_w[i].copy_((1.0 + 0.3 * torch.randn(net.ln_w[i].shape, generator=g)).cuda())
            net.ln_b[i].copy_((0.2 * torch.randn(net.ln_b[i].shape, generator=g)).cuda())
        for b in net.biases:
            b.add_((0.3 * torch.randn(b.shape, generator=g)).cuda())
    return actors


def _check(actors, env, P, training, seed):
    E, K = env.E, env.K
    mask = env.out["mask"]
    u = torch.rand((K, E, N_ACTIONS), device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed))
    logits_k = torch.full((K, E, N_ACTIONS), float("nan"), device="cuda")
    a_k, p_k = actors.act_env(env, mask, training, uniform=u, logits_out=logits_k, patch=P)
    win = env.obs_patch(P)                                 # [K, E, P, P]
    logits_r = actors(win)
    z = logits_r - torch.log(-torch.log(u + 1e-20) + 1e-20) if training else logits_r
    probs_r = torch.softmax(z, dim=-1)
    bits = (mask.t().to(torch.int32).unsqueeze(-1) >> torch.arange(N_ACTIONS, device="cuda")) & 1
    pm_r = torch.where(bits.bool(), probs_r, torch.zeros((), device="cuda"))
    torch.testing.assert_close(logits_k, logits_r, rtol=2e-4, atol=2e-4)
    torch.testing.assert_close(p_k, probs_r, rtol=0, atol=2e-5)
    top2 = pm_r.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1] > 1e-4).t()
    want = pm_r.argmax(-1).t().to(torch.int32)
    assert bool(clear.float().mean() > 0.5)
    assert torch.equal(a_k[clear], want[clear])
    assert bool(((mask.long() >> a_k.long()) & 1).all())
    return a_k


@pytest.mark.parametrize("scen,E,P,fear", [("grid32", 4096, 11, True), ("grid32", 1000, 8, False),
                                           ("grid64_n8", 2000, 16, False), ("level3", 64, 5, True),
                                           ("level3", 33, 40, False)])
def test_fused_patch_act_matches_torch_fp32_over_a_rollout(scen, E, P, fear):
    sc = S.builtin(scen)
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=5, max_steps=20, obs=False)
    actors = _actors(sc.K, P, seed=3)
    env.reset()
    _check(actors, env, P, training=True, seed=0)  # reset encoding (0.5 agents, 9.5 / 9 apples)
    for t in range(30):  # step encoding, relabels, eaten apples, auto-resets (20-step cap)
        a = actors.act_env(env, env.out["mask"], training=(t % 2 == 0), seed=1, counter=t, patch=P)[0]
        env.step(a)
        _check(actors, env, P, training=(t % 3 != 0), seed=t + 1)
    env.close()


def test_fused_patch_act_at_65536_envs():
    sc = S.builtin("grid64_n8")
    P = 16
    env = VecGridEnv(sc, num_envs=65536, fear=False, seed=8, max_steps=30, obs=False)
    actors = _actors(sc.K, P, seed=9)
    env.reset()
    for t in range(6):
        env.step()
    _check(actors, env, P, training=True, seed=77)
    env.close()


def test_fused_patch_rollout_matches_torch_rollout_without_noise():
    """Rollout(patch=P) fused == the PyTorch actor on the windows, step for step in eval mode (no
    noise): the same trajectories (so the same actions; no near-ties expected with random
    weights) and ring contents."""
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    E, P = 1024, 11
    envs = [VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=3, obs=False) for _ in range(2)]
    actors = _actors(sc.K, P, seed=5)
    ros = [Rollout(envs[0], actors, replay_slots=4, training=False, patch=P),
           Rollout(envs[1], actors, replay_slots=4, training=False, patch=P, fused=False)]
    assert ros[0].fused and not ros[1].fused
    for ro in ros:
        ro.reset()
    for t in range(25):
        r0, r1 = ros[0].step(), ros[1].step()
        assert torch.equal(r0.shaped, r1.shaped) and torch.equal(r0.done, r1.done), t
        ros[0].fence()  # (orders the window writer for the readers below)
        assert torch.equal(ros[0].replay.obs, ros[1].replay.obs), t
        torch.testing.assert_close(ros[0].replay.probs, ros[1].replay.probs, rtol=0, atol=2e-5)
    for e in envs:
        e.close()


@pytest.mark.parametrize("scenario,P", [("grid32", 11), ("grid64_n8", 16)])
def test_async_window_writer_equals_sync(scenario, P):
    """Rollout(patch=P) with the window writer on a side stream (patch_async=True; GW_PATCH_ASYNC=1) ==
    the same rollout with the writer on the caller's stream: every ring slot (windows, terminal
    windows, probs, rewards, dones) after fence(), training mode (Philox noise), a ragged E."""
    from marlnav.rollout import Rollout
    sc = S.builtin(scenario)
    E = 1000
    envs = [VecGridEnv(sc, num_envs=E, fear=scenario == "grid32", fear_weight=-5.0, seed=9, max_steps=20,
                       obs=False) for _ in range(2)]
    actors = _actors(sc.K, P, seed=8) if scenario == "grid32" else MultiAgentActors(sc.K, P, P, "cnn", device="cuda", seed=8)
    ros = [Rollout(envs[0], actors, replay_slots=5, training=True, seed=4, patch=P, patch_async=True),
           Rollout(envs[1], actors, replay_slots=5, training=True, seed=4, patch=P, patch_async=False)]
    assert ros[0].patch_async and not ros[1].patch_async
    for ro in ros:
        ro.reset()
    for t in range(40):
        for ro in ros:
            ro.step()
        if t % 7 == 6 or t == 39:
            ros[0].fence()
            a, b = ros[0].replay, ros[1].replay
            assert torch.equal(a.obs, b.obs) and torch.equal(a.probs, b.probs), t
            assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), t
            done = b.done.bool()
            assert torch.equal(a.final_obs.transpose(1, 2)[done], b.final_obs.transpose(1, 2)[done]), t
    assert int(ros[1].replay.done.sum()) > 0  # terminal windows were exercised
    for e in envs:
        e.close()


def test_cnn_head_on_windows_matches_conv2d_at_65536_envs():
    """The configs/cnn.yaml head on 16 x 16 windows (bench.py --config c4patch: the PyTorch forward
    as per-patch GEMMs, CNNActor._forward_patch_gemm) == nn.Conv2d -> flatten -> MLP on the same
    windows, fp32, 65,536 envs of the 64 x 64 / N = 8 grid.  Tolerance 1e-4 relative + 1e-4
    absolute on the logits (GEMM vs convolution summation order)."""
    sc = S.builtin("grid64_n8")
    P = 16
    env = VecGridEnv(sc, num_envs=65536, fear=False, seed=12, max_steps=30, obs=False)
    actors = MultiAgentActors(sc.K, P, P, "cnn", device="cuda", seed=4)
    env.reset()
    for _ in range(5):
        env.step()
    win = env.obs_patch(P)                                   # [K, E, P, P]
    with torch.no_grad():
        for k in range(sc.K):
            m = actors.nets[k]
            assert m.patchify
            x = win[k].unsqueeze(1)
            got = m(x)
            ref = m.mlp(m.conv(x).flatten(1))
            torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    env.close()
