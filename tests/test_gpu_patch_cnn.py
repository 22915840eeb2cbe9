"""The configs/cnn.yaml head on each RL agent's P x P egocentric window as one fused HIP path
(gw_patch_cnn_act; X1, not a reference format) against the PyTorch fp32 head in its nn.Conv2d form
(maddpg/agent.py:94-100 with configs/cnn.yaml:2-6 at input P x P) on the windows
``VecGridEnv.obs_patch(P)`` writes (themselves == -1-padded crops of the oracle-pinned full obs,
tests/test_gpu_obs_patch.py).

Layer 1 = the centre cell's table row (b + Linear-1 of the base window: the map under the window
with the agent's usual own value at the centre) + Wl[:, Q] . (a2(Q) - a2_base(Q)) for each window
position Q the step's patched cells change, recomputed from the obs descriptors.  That differs
from torch only in f32 summation order (a 1024-long Linear-1 dot as table + deltas).  Tolerances
(as tests/test_gpu_cnn_actor.py): logits |d| <= 5e-4 + 5e-4 |x|; probs |d| <= 5e-5; actions equal
wherever the best masked probability leads the runner-up by more than 1e-3.
"""
import pytest
import torch

from marlnav import scenario as S
from marlnav.actor import MultiAgentActors, N_ACTIONS
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _actors(K, P, seed):
    actors = MultiAgentActors(K, P, P, arch="cnn", device="cuda", seed=seed)
    g = torch.Generator(device="cpu").manual_seed(seed + 100)
    with torch.no_grad():  # larger conv biases: more ReLUs change state under a patched cell
        for n in actors.nets:
            for conv in (n.conv[0], n.conv[2]):
                conv.bias.add_((0.2 * torch.randn(conv.bias.shape, generator=g)).cuda())
    return actors


def _dense_logits(actors, win):
    """torch fp32 reference: nn.Conv2d -> ReLU -> nn.Conv2d -> ReLU -> flatten -> MLP per agent."""
    with torch.no_grad():
        return torch.stack([n.mlp(n.conv(win[k].unsqueeze(1)).flatten(1)) for k, n in enumerate(actors.nets)])


def _check(actors, env, P, training, seed):
    E, K = env.E, env.K
    mask = env.out["mask"]
    u = torch.rand((K, E, N_ACTIONS), device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed))
    logits_k = torch.full((K, E, N_ACTIONS), float("nan"), device="cuda")
    a_k, p_k = actors.act_env(env, mask, training, uniform=u, logits_out=logits_k, patch=P)
    logits_r = _dense_logits(actors, env.obs_patch(P))
    z = logits_r - torch.log(-torch.log(u + 1e-20) + 1e-20) if training else logits_r
    probs_r = torch.softmax(z, dim=-1)
    bits = (mask.t().to(torch.int32).unsqueeze(-1) >> torch.arange(N_ACTIONS, device="cuda")) & 1
    pm_r = torch.where(bits.bool(), probs_r, torch.zeros((), device="cuda"))
    torch.testing.assert_close(logits_k, logits_r, rtol=5e-4, atol=5e-4)
    torch.testing.assert_close(p_k, probs_r, rtol=0, atol=5e-5)
    top2 = pm_r.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1] > 1e-3).t()
    want = pm_r.argmax(-1).t().to(torch.int32)
    assert bool(clear.float().mean() > 0.25)  # (the action check is not vacuous)
    assert torch.equal(a_k[clear], want[clear])
    assert bool(((mask.long() >> a_k.long()) & 1).all())
    return a_k


@pytest.mark.parametrize("scen,E,P,fear,variant", [("grid64_n8", 2000, 16, False, 0), ("grid32", 4096, 16, True, 0),
                                                   ("grid32", 777, 8, False, 0), ("level3", 64, 12, True, 0),
                                                   ("level3_single", 33, 4, False, 1),
                                                   ("level3_single", 50, 16, False, 1)])
def test_fused_patch_cnn_matches_conv2d_over_a_rollout(scen, E, P, fear, variant):
    sc = S.builtin(scen)
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=5, max_steps=20, obs=False, variant=variant)
    actors = _actors(sc.K, P, seed=3)
    env.reset()
    _check(actors, env, P, training=True, seed=0)  # reset encoding (0.5 agents, 9.5 / 9 apples)
    for t in range(30):  # step encoding, relabels, eaten apples, auto-resets (20-step cap)
        a = actors.act_env(env, env.out["mask"], training=(t % 2 == 0), seed=1, counter=t, patch=P)[0]
        env.step(a)
        _check(actors, env, P, training=(t % 3 != 0), seed=t + 1)
    env.close()


def test_fused_patch_cnn_at_65536_envs():
    """bench.py --config c4patch's size (64 x 64, N = 8, K = 2, 65,536 envs, P = 16)."""
    sc = S.builtin("grid64_n8")
    P = 16
    env = VecGridEnv(sc, num_envs=65536, fear=False, seed=8, max_steps=30, obs=False)
    actors = _actors(sc.K, P, seed=9)
    env.reset()
    _check(actors, env, P, training=True, seed=70)
    for t in range(6):
        env.step()
    _check(actors, env, P, training=True, seed=77)
    env.close()


def test_fused_patch_cnn_follows_weight_updates():
    """A parameter change (torch in-place op) re-derives the tables before the next act."""
    sc = S.builtin("grid32")
    P = 16
    env = VecGridEnv(sc, num_envs=512, fear=False, seed=2, obs=False)
    actors = _actors(sc.K, P, seed=1)
    env.reset()
    env.step()
    _check(actors, env, P, training=False, seed=1)
    with torch.no_grad():
        for n in actors.nets:
            n.conv[0].weight.mul_(-1.5)
            n.mlp[0].bias.add_(0.5)
    _check(actors, env, P, training=False, seed=2)
    env.close()


def test_fused_patch_cnn_rollout_matches_torch_rollout_without_noise():
    """Rollout(patch=P) with the CNN head: fused == the PyTorch head on the windows, step for step
    in eval mode (no noise): the same trajectories and ring contents."""
    from marlnav.rollout import Rollout
    sc = S.builtin("grid64_n8")
    E, P = 1024, 16
    envs = [VecGridEnv(sc, num_envs=E, fear=False, seed=3, obs=False) for _ in range(2)]
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
        torch.testing.assert_close(ros[0].replay.probs, ros[1].replay.probs, rtol=0, atol=5e-5)
    for e in envs:
        e.close()


def test_write_list_equals_obs_patch_and_act():
    """gw_patch_cnn_write_list == gw_obs_patch (windows and terminal windows, bit for bit) and,
    with gw_patch_cnn_act_listed, == gw_patch_cnn_act (actions and probabilities bit for bit),
    over a rollout with auto-resets; a refused second listing while one is pending, a listing
    consumed by the self-listing act, and a weight change after the listing (the act then
    re-derives and lists itself), included."""
    sc = S.builtin("grid64_n8")
    P, E = 16, 3000
    env = VecGridEnv(sc, num_envs=E, fear=False, seed=4, max_steps=12, obs=False)
    actors = _actors(sc.K, P, seed=6)
    env.reset()
    actors.act_env(env, env.out["mask"], True, seed=2, counter=0, patch=P)  # derives the workspace
    K = sc.K
    outs = [torch.full((K, E, P, P), float("nan"), device="cuda") for _ in range(4)]
    for t in range(30):
        assert actors.patch_cnn_write_list(env, P, outs[0], outs[1])
        if t % 7 == 3:  # no second listing while one is pending (its counts would add up)
            assert not actors.patch_cnn_write_list(env, P, outs[0], outs[1])
        env.obs_patch(P, final=True, out=outs[2], final_out=outs[3])
        assert torch.equal(outs[0], outs[2]), t
        assert torch.equal(torch.nan_to_num(outs[1], nan=7.0), torch.nan_to_num(outs[3], nan=7.0)), t
        if t == 17:  # a weight change after the listing: act_env re-derives and lists itself
            with torch.no_grad():
                actors.nets[1].mlp[0].bias.add_(0.01)
        if t % 5 == 4:  # the listing consumed by the self-listing act (gw_patch_cnn_act zeroes first)
            a1, p1 = [x.clone() for x in actors.act_env(env, env.out["mask"], True, seed=2, counter=t, patch=P)]
        else:
            a1, p1 = [x.clone() for x in actors.act_env(env, env.out["mask"], True, seed=2, counter=t, patch=P,
                                                         listed=True)]
        a0, p0 = actors.act_env(env, env.out["mask"], True, seed=2, counter=t, patch=P)
        assert torch.equal(a0, a1) and torch.equal(p0, p1), t
        env.step(a0)
    env.close()


@pytest.mark.parametrize("graph", [False, True])
def test_rollout_write_list_equals_separate_writer_and_act(graph, monkeypatch):
    """Rollout with the CNN head on windows (default: the windows and the next act's listing in one
    launch) == the separate writer and act (GW_CNN_WRITE_LIST=0): identical ring contents over a
    training rollout with auto-resets and a Rollout.reset in between, eager and as ring-phase
    graphs."""
    from marlnav.rollout import Rollout
    sc = S.builtin("grid64_n8")
    E, P, n = 2048, 16, 4
    actors = _actors(sc.K, P, seed=7)
    rings = []
    for fused in ("1", "0"):
        monkeypatch.setenv("GW_CNN_WRITE_LIST", fused)
        env = VecGridEnv(sc, num_envs=E, fear=False, seed=9, max_steps=12, obs=False)
        ro = Rollout(env, actors, replay_slots=8, training=True, seed=3, patch=P)
        assert ro._cnn_list == (fused == "1")
        ro.reset()
        for _ in range(5):
            ro.step()
        ro.reset()  # a listing left by the last step is not used after the reset
        for _ in range(3):
            ro.step()
        if graph:
            g = ro.capture(n)
            for _ in range(3):
                g.replay()
        else:
            for _ in range(3 * n):
                ro.step()
        ro.fence()
        torch.cuda.synchronize()
        rings.append((ro.replay.obs.clone(), ro.replay.probs.clone(), ro.replay.reward.clone(),
                      ro.replay.done.clone(), torch.nan_to_num(ro.replay.final_obs, nan=7.0)))
        env.close()
    for x, y in zip(*rings):
        assert torch.equal(x, y)
