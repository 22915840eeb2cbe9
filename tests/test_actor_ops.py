"""Fused get_action (gw_actor_act, include/actor_ops.h) against the PyTorch fp32 actor on the
dense observations the env wrote.

The kernel evaluates the first layer from the obs descriptors (c1 = b1 + map.W1 plus one W1 row
per patched cell) and layers 2-3 on f32 MFMA, so it differs from torch's dense GEMMs only in
f32 summation order.  Tolerances (stated here, float32 path): logits |d| <= 2e-4 + 2e-4 |x|;
probs |d| <= 2e-5; actions equal wherever the best masked probability leads the runner-up by
more than 1e-4 (a closer race may legitimately resolve either way).  The Gumbel uniforms are
passed in explicitly so both paths see the same noise; Philox-noise mode is checked for law
(mask respected, distribution, determinism per counter).
"""
import pytest
import torch

from marlnav import scenario as S
from marlnav.actor import MultiAgentActors, N_ACTIONS
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _actors(sc, seed, layer_norm=True):
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=seed)
    net = actors.net
    net.layer_norm = layer_norm
    g = torch.Generator(device="cpu").manual_seed(seed + 100)
    with torch.no_grad():  # non-trivial LayerNorm affine and biases
        for i in range(2):
            net.ln_w[i].copy_((1.0 + 0.3 * torch.randn(net.ln_w[i].shape, generator=g)).cuda())
            net.ln_b[i].copy_((0.2 * torch.randn(net.ln_b[i].shape, generator=g)).cuda())
    return actors


def _reference(actors, env, mask, training, u, tau=1.0):
    """MultiAgentActors.act restated with explicit uniforms (torch fp32, dense obs)."""
    logits = actors(env.out["obs"])
    z = logits - torch.log(-torch.log(u + 1e-20) + 1e-20) if training else logits
    probs = torch.softmax(z / tau, dim=-1)
    bits = (mask.t().to(torch.int32).unsqueeze(-1) >> torch.arange(N_ACTIONS, device=mask.device)) & 1
    pm = torch.where(bits.bool(), probs, torch.zeros((), device=probs.device))
    return logits, probs, pm


def _check(actors, env, training, seed=0):
    E, K = env.E, env.K
    mask = env.out["mask"]
    u = torch.rand((K, E, N_ACTIONS), device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed))
    logits_k = torch.full((K, E, N_ACTIONS), float("nan"), device="cuda")
    a_k, p_k = actors.act_env(env, mask, training, uniform=u, logits_out=logits_k)
    logits_r, probs_r, pm_r = _reference(actors, env, mask, training, u)
    torch.testing.assert_close(logits_k, logits_r, rtol=2e-4, atol=2e-4)
    torch.testing.assert_close(p_k, probs_r, rtol=0, atol=2e-5)
    top2 = pm_r.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1] > 1e-4).t()  # [E, K]
    want = pm_r.argmax(-1).t().to(torch.int32)
    assert bool(clear.float().mean() > 0.5)
    assert torch.equal(a_k[clear], want[clear])
    allowed = (mask.long() >> a_k.long()) & 1
    assert bool(allowed.all())
    return a_k


@pytest.mark.parametrize("scen,E,fear", [("grid32", 4096, True), ("grid64_n8", 1000, False), ("level3", 33, True),
                                         ("level3", 1, False)])
def test_fused_act_matches_torch_fp32_over_a_rollout(scen, E, fear):
    sc = S.builtin(scen)
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=5, max_steps=20)
    actors = _actors(sc, seed=3)
    env.reset()
    _check(actors, env, training=True, seed=0)  # reset encoding (0.5 agents, 9.5 / 9 apples)
    for t in range(30):  # step encoding, relabels, eaten apples, auto-resets (20-step cap)
        a = actors.act_env(env, env.out["mask"], training=(t % 2 == 0), seed=1, counter=t)[0]
        env.step(a)
        _check(actors, env, training=(t % 3 != 0), seed=t + 1)
    env.close()


def test_fused_act_without_layer_norm_and_single_agent_variant():
    sc = S.builtin("level3_single")
    env = VecGridEnv(sc, num_envs=300, fear=False, seed=9, variant="single", max_steps=15)
    actors = _actors(sc, seed=4, layer_norm=False)
    env.reset()
    for t in range(20):
        a = _check(actors, env, training=True, seed=100 + t)
        env.step(a)
    env.close()


def test_fused_act_philox_noise_law():
    sc = S.builtin("grid32")
    E = 8192
    env = VecGridEnv(sc, num_envs=E, fear=False, seed=1)
    actors = _actors(sc, seed=7)
    with torch.no_grad():  # zero weights: logits = 0, so the action is the argmax of pure Gumbel noise
        actors.net.flat_params().zero_()
    env.reset()
    mask = env.out["mask"]
    a1, p1 = actors.act_env(env, mask, True, seed=11, counter=0)
    a1, p1 = a1.clone(), p1.clone()
    a2, p2 = actors.act_env(env, mask, True, seed=11, counter=0)
    assert torch.equal(a1, a2) and torch.equal(p1, p2)  # deterministic per (seed, counter)
    a3, _ = actors.act_env(env, mask, True, seed=11, counter=1)
    assert not torch.equal(a1, a3)
    torch.testing.assert_close(p1.sum(-1), torch.ones((sc.K, E), device="cuda"), rtol=0, atol=1e-5)
    assert bool(((mask.long() >> a1.long()) & 1).all())
    # uniform over the allowed actions: over the (env, agent) pairs with the most common mask,
    # each allowed action ~ 1 / (allowed count)
    m = mask.long()
    mode = int(torch.mode(m.flatten()).values)
    sel = m == mode
    counts = torch.bincount(a1[sel].long(), minlength=9).float()
    n, allowed_n = counts.sum(), bin(mode).count("1")
    assert n > 500 and allowed_n >= 2
    for a in range(9):
        if (mode >> a) & 1:
            q = 1 / allowed_n
            assert abs(float(counts[a] / n) - q) < 5 * (q * (1 - q) / float(n)) ** 0.5, (a, counts)
        else:
            assert counts[a] == 0
    a_eval, p_eval = actors.act_env(env, mask, False)
    torch.testing.assert_close(p_eval, torch.full_like(p_eval, 1 / 9))
    assert bool((a_eval == 0).all())  # all ties: first maximum (Stay), as torch.argmax
    env.close()


def test_rollout_fused_matches_unfused_without_noise():
    """Rollout(fused) == Rollout(unfused) step for step in eval mode (no noise): same actions
    (up to near-ties, none expected with random weights), same replay contents."""
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    E = 1024
    envs = [VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=3, debug=True) for _ in range(2)]
    actors = _actors(sc, seed=5)
    ros = [Rollout(envs[0], actors, replay_slots=3, training=False, fused=True),
           Rollout(envs[1], actors, replay_slots=3, training=False, fused=False)]
    for ro in ros:
        ro.reset()
    assert ros[0].fused and not ros[1].fused
    same = 0
    for t in range(25):
        r0, r1 = ros[0].step(), ros[1].step()
        if torch.equal(r0.actions, r1.actions):
            same += 1
        else:
            break
        assert torch.equal(r0.obs, r1.obs) and torch.equal(r0.shaped, r1.shaped)
        torch.testing.assert_close(ros[0].replay.probs, ros[1].replay.probs, rtol=0, atol=2e-5)
    assert same == 25
    for e in envs:
        e.close()


def test_fused_act_sees_every_weight_update():
    """The workspace (c1, W2/W3 images) is re-derived after the HIP optimizer, a graph replay of
    the update, a checkpoint load and a plain in-place torch write."""
    from marlnav.maddpg import MADDPG
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=512, fear=False, seed=2)
    learner = MADDPG(sc.K, sc.H, sc.W, device="cuda", seed=1, capturable=True)
    ro = Rollout(env, learner.actors, replay_slots=8, training=True, seed=3)
    ro.reset()
    for _ in range(4):
        ro.step()

    def agree():
        u = torch.rand((sc.K, env.E, N_ACTIONS), device="cuda")
        lk = torch.empty((sc.K, env.E, N_ACTIONS), device="cuda")
        learner.actors.act_env(env, env.out["mask"], True, uniform=u, logits_out=lk)
        torch.testing.assert_close(lk, learner.actors(ro._obs_now()), rtol=2e-4, atol=2e-4)  # the ring slot

    agree()
    learner.learn_from(ro.replay)  # FlatAdam (HIP) on the actors
    agree()
    learner.capture(ro.replay)
    learner.replay_learn()         # graph replay
    agree()
    learner.capture(ro.replay, actor_env=env)  # the graph ends with the workspace derivation
    assert learner._prep_env is env
    calls = []
    eager = learner.actors._prepare
    learner.actors._prepare = lambda *a: (calls.append(1), eager(*a))
    for _ in range(2):
        learner.replay_learn()
        agree()
    assert not calls  # act_env did not derive the workspace again
    learner.actors._prepare = eager
    sd = {k: v.clone() for k, v in learner.state_dict().items()}
    with torch.no_grad():
        learner.actors.net.weights[1].mul_(-1.5)  # plain in-place write through a layer view
    agree()
    learner.load_state_dict(sd)   # checkpoint load
    agree()
    env.close()


@pytest.mark.parametrize("variant", ["4", "2"])
def test_fused_act_layer2_precision(variant, monkeypatch):
    """Logits of the fused op (GW_ACT_V=4: layer 2 as bf16x3 MFMA products, the default; 2: exact
    f32 MFMA) against a float64 forward of the same weights: both within f32 rounding noise."""
    monkeypatch.setenv("GW_ACT_V", variant)
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=2048, fear=True, fear_weight=-5.0, seed=6)
    actors = _actors(sc, seed=11)
    env.reset()
    for _ in range(3):
        env.step()
    logits = torch.empty((sc.K, env.E, N_ACTIONS), device="cuda")
    actors.act_env(env, env.out["mask"], False, logits_out=logits)
    net = actors.net
    x = env.out["obs"].reshape(sc.K, env.E, -1).double()
    h = x
    for i in range(3):
        h = torch.bmm(h, net.weights[i].double()) + net.biases[i].double().reshape(sc.K, 1, -1)
        if i < 2:
            if net.layer_norm:
                h = torch.nn.functional.layer_norm(h, (h.shape[-1],), eps=1e-5)
                h = h * net.ln_w[i].double().reshape(sc.K, 1, -1) + net.ln_b[i].double().reshape(sc.K, 1, -1)
            h = torch.relu(h)
    err = (logits.double() - h).abs().max().item()
    assert err < 2e-5, err
    env.close()


@pytest.mark.parametrize("E", [4096, 777, 20000])
def test_fused_act_block_shape_does_not_change_results(E, monkeypatch):
    """The actor's block shape (4 / 8 / 12 / 16 waves: GW_ACT_WAVES) does not change the results:
    each wave evaluates whole 16-env tiles, so logits, probabilities and actions (Philox noise)
    are bit for bit the same, and every launch writes every output (sentinel-filled buffers)."""
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=E, fear=False, seed=12)
    actors = _actors(sc, seed=13)
    env.reset()
    env.step()
    out = {}
    for sched in ("static",):
        for w in ("4", "8", "12", "16"):
            monkeypatch.setenv("GW_ACT_WAVES", w)
            for rep in range(2):
                lk = torch.full((sc.K, E, N_ACTIONS), float("nan"), device="cuda")
                a = torch.full((E, sc.K), -7, dtype=torch.int32, device="cuda")
                pr = torch.full((sc.K, E, N_ACTIONS), float("nan"), device="cuda")
                actors.act_env(env, env.out["mask"], True, seed=5, counter=9, logits_out=lk, actions_out=a,
                               probs_out=pr)
                assert not torch.isnan(lk).any() and not torch.isnan(pr).any() and bool((a >= 0).all())
                out[(sched, w, rep)] = (a, pr, lk)
    ref = out[("static", "16", 0)]
    for key, v in out.items():
        for x, y in zip(v, ref):
            assert torch.equal(x, y), key
    env.close()
