"""The descriptor learner (gw_maddpg_desc_update, include/learner_ops.h): one MADDPG update
(agilerl MADDPG.learn via maddpg/agent.py:199-224) on the replay ring of obs descriptors in four
launches, layer 1 as the map part c1 = b1 + map . W1 plus the patched cells, the W1 gradient as
map (x) colsum(dZ1) plus the patched cells' terms, Adam and the soft updates inside.

Pinned against the dense fused update (gw_maddpg_critic_grads / _actor_grads + flat Adam + soft
update; itself pinned to the torch autograd composition in tests/test_maddpg_fused.py) on the
SAME rows and Gumbel uniforms (both draw them with the same Philox keys and counters), and
against the autograd composition on the dense rows of the sampled transitions: every gradient
tensor within 1e-5 relative L2, the updated parameters within f32 rounding, the losses.  The
update is deterministic: recorded launches == a graph replay == eager calls, bit for bit."""
import pytest
import torch

from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _setup(E=512, fear=True, scen="grid32", steps=7, seed=7, cap=10):
    from marlnav.maddpg import MADDPG
    from marlnav.rollout import Rollout
    sc = S.builtin(scen)
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, stats=True, seed=seed, max_steps=cap)
    m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
    ro = Rollout(env, m.actors, replay_slots=16, training=True, seed=4, obs_async=True, desc_ring=True)
    ro.reset()
    for _ in range(steps):
        ro.step()
    ro.fence()
    return sc, env, m, ro


def _dense_batch(rp, idx):
    """The sampled transitions' dense rows (state [K,B,H,W], probs, reward [B,K], next state, term)."""
    tr, env = idx[:, 0].long(), idx[:, 1].long()
    nx = (tr + 1) % rp.S
    done = rp.done[tr, env].bool()
    st = rp.obs[tr, :, env].permute(1, 0, 2, 3).float()
    ns = torch.where(done[None, :, None, None], rp.final_obs[tr, :, env].permute(1, 0, 2, 3),
                     rp.obs[nx, :, env].permute(1, 0, 2, 3)).float()
    return st, rp.probs[tr, :, env].permute(1, 0, 2).contiguous(), rp.reward[tr, env], ns, rp.term[tr, env]


def _grads(m):
    return {"critic": m.critics.flat_params().grad.clone(), "actor": m.actors.net.flat_params().grad.clone()}


def _rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _per_tensor(net, flat_a, flat_b):
    """relative L2 of every parameter tensor's slice of two flat buffers of ``net``'s layout"""
    base = net.flat_params().data_ptr()
    out = {}
    for name, t in net.named_parameters():
        o = (t.data_ptr() - base) // 4
        n = t.numel()
        out[name] = _rel(flat_a[o:o + n], flat_b[o:o + n])
    return out


@pytest.mark.parametrize("scen,E,fear,B", [("grid32", 512, True, 128), ("level3", 300, False, 128),
                                           ("grid64_n8", 256, True, 128),
                                           # dZ1 rows beyond the W1 blocks' LDS copy (B > 128); a small batch
                                           ("grid32", 512, True, 256), ("grid64_n8", 256, True, 48)])
def test_desc_update_equals_dense_fused_update(scen, E, fear, B):
    sc, env, m, ro = _setup(E=E, fear=fear, scen=scen)
    from marlnav.maddpg import MADDPG
    m.batch_size = B
    m2 = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True, batch_size=B)
    assert torch.equal(m2.critics.flat_params(), m.critics.flat_params())
    rp = ro.replay
    assert m.desc_capable(rp)
    la, lc = m.learn_desc(rp)
    rec = m.desc_records(rp)
    # the dense fused update on the same rows (its gather draws them with the same Philox key and count)
    batch = m2._sample(rp)
    la2, lc2 = m2.learn(*batch)
    torch.cuda.synchronize()
    g1, g2 = _grads(m), _grads(m2)
    for net, which in ((m.critics, "critic"), (m.actors.net, "actor")):
        errs = _per_tensor(net, g1[which], g2[which])
        assert max(errs.values()) < 1e-5, (which, errs)
    assert torch.allclose(lc, lc2, rtol=1e-5, atol=1e-6) and torch.allclose(la, la2, rtol=1e-5, atol=1e-6)
    for a, b in ((m.critics, m2.critics), (m.actors.net, m2.actors.net), (m.critic_targets, m2.critic_targets),
                 (m.actor_targets.net, m2.actor_targets.net)):
        # one Adam step: the step direction m / sqrt(v) divides out the gradient's scale, so an
        # element whose gradient differs in its last bits moves by lr * (that relative difference)
        # (measured 1.5e-6 at 64 x 64 / N = 8)
        assert _rel(a.flat_params().detach(), b.flat_params().detach()) < 1e-5
    # the rows it recorded are the transitions the dense gather sampled
    B = m.batch_size
    assert rec["idx"].shape == (B, 2)
    assert m.opt_critic.count[0].item() == m2.opt_critic.count[0].item() == 1
    assert m.opt_actor.count[0].item() == m2.opt_actor.count[0].item() == 1
    env.close()


def test_desc_update_equals_autograd_composition():
    """Against the torch autograd composition (GW_FUSED_LEARN=0's learner) on the dense rows of
    the transitions the descriptor learner sampled, with its Gumbel uniforms: every gradient tensor
    within 1e-5 relative L2."""
    sc, env, m, ro = _setup()
    from marlnav.maddpg import MADDPG
    m3 = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
    m3.fused = False
    rp = ro.replay
    m.learn_desc(rp)
    rec = m.desc_records(rp)
    st, ac, rw, ns, dn = _dense_batch(rp, rec["idx"])
    m3.learn(st, ac, rw, ns, dn, rec["u_next"], rec["u_cur"])
    torch.cuda.synchronize()
    g1, g3 = _grads(m), _grads(m3)
    for net, which in ((m.critics, "critic"), (m.actors.net, "actor")):
        errs = _per_tensor(net, g1[which], g3[which])
        assert max(errs.values()) < 1e-5, (which, errs)
    env.close()


def test_desc_update_replays_bit_for_bit():
    """Eager calls, recorded launches and a HIP-graph replay of the descriptor learner give the same
    weights bit for bit after several updates interleaved with env steps."""
    from marlnav.maddpg import MADDPG
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    states = []
    for mode in ("eager", "launches", "graph"):
        env = VecGridEnv(sc, num_envs=512, fear=True, fear_weight=-5.0, stats=True, seed=7, max_steps=10)
        m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=3, capturable=True)
        ro = Rollout(env, m.actors, replay_slots=16, training=True, seed=4, obs_async=True, desc_ring=True)
        ro.reset()
        for t in range(12):
            ro.step()
            if t < 2:
                continue
            ro.learn_fence()
            if mode == "eager":
                m.learn_desc(ro.replay)
            else:
                if m._graph is None:
                    m.capture(ro.replay, actor_env=env, launches=mode == "launches", warmup=1)
                else:
                    m.replay_learn()
        torch.cuda.synchronize()
        if mode == "launches":
            calls = [c[0] for c in m._launches.calls]
            # one call; the fused actor's workspace comes from the update itself (no prepare launches)
            assert calls == ["gw_maddpg_desc_update_img"], calls
        states.append({k: v.clone() for k, v in m.state_dict().items()})
        env.close()
    for s in states[1:]:
        for k in states[0]:
            assert torch.equal(states[0][k], s[k]), k


def test_desc_learner_primes_after_a_load():
    """Weights loaded (or stepped by the dense path) after the descriptor learner's c1 partial sums
    were derived must not be used with stale sums: the next update re-derives them, so it equals
    an update of a fresh learner holding the same weights."""
    from marlnav.maddpg import MADDPG
    sc, env, m, ro = _setup()
    rp = ro.replay
    m.learn_desc(rp)
    m.learn(*m._sample(rp))                 # a dense update: weights change outside the learner
    sd, osd = m.state_dict(), m.optim_state_dict()
    m2 = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=11, capturable=True)
    m2.load_state_dict({k: v.clone() for k, v in sd.items()})
    m2.load_optim_state_dict({k: v.clone() for k, v in osd.items()})
    m2._draw_key = m._draw_key
    m.learn_desc(rp)
    m2.learn_desc(rp)
    torch.cuda.synchronize()
    for a, b in ((m.critics, m2.critics), (m.actors.net, m2.actors.net)):
        assert torch.equal(a.flat_params(), b.flat_params())
    env.close()


def test_desc_update_leaves_the_fused_actor_workspace():
    """gw_maddpg_desc_update_img (learn_desc with the env the fused actor acts on) leaves the fused
    actor's row slices and W2 / W3 operand images bit for bit as gw_actor_prepare derives them
    from the updated weights, and act_env then runs without a prepare."""
    sc, env, m, ro = _setup()
    rp = ro.replay
    st = m.actors._fast
    assert st is not None and st["env"] is env
    m.learn_desc(rp, actor_env=env)
    assert st["key"] == m.actors._ws_key()  # marked prepared: the next act_env derives nothing
    torch.cuda.synchronize()
    ws_learner = st["ws"].clone()
    m.actors._prepare(env, st)
    torch.cuda.synchronize()
    K, HW, HID = sc.K, sc.H * sc.W, 128
    w2img, w3img, w2bimg = HID * HID, 8 * 4 * 9 * 4, 3 * 8 * 4 * 64 * 4
    o_w2 = K * HID                      # (c1 first: the learner leaves it, gw_actor_act sums the slices)
    o_end = K * (HID + w2img + w3img + w2bimg) + K * ((HW + 31) // 32) * HID
    a, b = ws_learner[o_w2:o_end].view(torch.int32), st["ws"][o_w2:o_end].view(torch.int32)
    assert torch.equal(a, b), int((a != b).sum())
    env.close()
