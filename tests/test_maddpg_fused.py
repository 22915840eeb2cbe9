"""The fused MADDPG update (csrc/maddpg_ops.hip: gw_maddpg_critic_grads / gw_maddpg_actor_grads,
the default GPU learner) against the torch-autograd composition of the same update
(marlnav/maddpg.py with GW_FUSED_LEARN=0, itself pinned to the per-agent agilerl-style loop in
tests/test_maddpg.py) and against that per-agent loop.

Tolerances.  The fused kernels sum in other orders than torch's GEMMs and LayerNorm (f32,
deterministic).  (1) One update's gradients: EVERY gradient tensor within 1e-5 relative L2 of
autograd's (measured: 2e-7 .. 6e-7, profiles/r3_learner), the losses within 1e-4 relative, the
target actions (x_next's slots) within 2e-6.  The bound is that tight because no ReLU input of
the batch lies within 1e-5 of zero (asserted from a float64 forward of every network the update
evaluates): a ReLU at the f32 rounding edge of its LayerNorm could take the other side in one of
the two and move one row's contribution by far more than rounding; such rows are masked (replaced
by a copy of a clean row of the batch, at most 2 of 128) before the comparison.  A negative check shows the
bound bites: scaling any single gradient tensor by (1 + 1e-4) fails it.  (2) Four updates
against the per-agent loop: losses within 1e-4 relative, every parameter tensor within 1e-5
relative L2 (measured worst 3.2e-7).  (3) A HIP-graph replay of the fused update equals the eager
fused update bit for bit (fixed orders).
"""
import pytest
import torch

from marlnav.maddpg import MADDPG

pytestmark = pytest.mark.gpu

K, H, W, B, LR = 2, 32, 32, 128, 1e-3


def _batch(g, B_=B):
    states = torch.randint(-1, 6, (K, B_, H, W), generator=g, device="cuda").float()
    next_states = torch.randint(-1, 6, (K, B_, H, W), generator=g, device="cuda").float()
    actions = torch.softmax(torch.randn((K, B_, 9), generator=g, device="cuda") * 2, -1)
    rewards = torch.randn((B_, K), generator=g, dtype=torch.float64, device="cuda") * 10
    dones = (torch.rand((B_, K), generator=g, device="cuda") < 0.2).to(torch.uint8)
    u_next = torch.rand((K, B_, 9), generator=g, device="cuda")
    u_cur = torch.rand((K, B_, 9), generator=g, device="cuda")
    return states, actions, rewards, next_states, dones, u_next, u_cur


def _pair(seed=3):
    ms = [MADDPG(K, H, W, lr_actor=LR, lr_critic=LR, gamma=0.98, tau=0.01, batch_size=B, device="cuda", seed=seed,
                 capturable=True) for _ in range(2)]
    assert ms[0].fused
    ms[1].fused = False
    g = torch.Generator(device="cuda").manual_seed(seed + 50)
    with torch.no_grad():  # targets apart from the online nets, non-trivial LayerNorm affines
        for m in ms:
            gg = torch.Generator(device="cuda").manual_seed(seed + 50)
            for net in (m.actor_targets.net, m.critic_targets):
                net.flat_params().add_(0.05 * torch.randn(net.flat_params().shape, device="cuda", generator=gg))
            for net in (m.actors.net, m.critics):
                for lw, lb in zip(net.ln_w, net.ln_b):
                    lw.add_(0.2 * torch.randn(lw.shape, device="cuda", generator=gg))
                    lb.add_(0.1 * torch.randn(lb.shape, device="cuda", generator=gg))
    del g
    return ms


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _grads(net):
    return [p.grad.detach().clone() for p in (net.weights[0], net.biases[0], net.ln_w[0], net.ln_b[0], net.weights[1],
                                              net.biases[1], net.ln_w[1], net.ln_b[1], net.weights[2], net.biases[2])]


GRAD_TOL = 1e-5  # relative L2 per gradient tensor
EDGE = 1e-5      # a ReLU input this close to 0 could flip between two f32 summation orders


def _relu_margin(net, x):
    """min |ReLU input| over the hidden layers of ``net`` on inputs x [K, B, in] (float64 forward:
    Linear -> LayerNorm(eps 1e-5) -> affine), and the rows [B] (bool) with an input within EDGE
    of zero."""
    h = x.double()
    lo, rows = float("inf"), torch.zeros(x.shape[1], dtype=torch.bool, device=x.device)
    with torch.no_grad():
        for i in range(net.n_layers - 1):
            z = torch.baddbmm(net.biases[i].double(), h, net.weights[i].double())
            mu = z.mean(-1, keepdim=True)
            a = (z - mu) / torch.sqrt(((z - mu) ** 2).mean(-1, keepdim=True) + 1e-5) * net.ln_w[i].double() + \
                net.ln_b[i].double()
            lo = min(lo, float(a.abs().min()))
            rows |= (a.abs() < EDGE).any(-1).any(0)
            h = torch.relu(a)
    return lo, rows


def _edge_rows(ref, st, ac, ns, un, uc, critic_after=None):
    """Rows of the batch where a network the update evaluates has a ReLU input within EDGE of zero:
    autograd's target actors, target critic, critic and actor before the update, and the critic
    after its Adam step (``critic_after``: the actor phase evaluates it on the mixed actions)."""
    from marlnav.maddpg import gumbel_softmax
    x = ref._critic_in(st, ac)
    with torch.no_grad():
        xt = ref._critic_in(ns, gumbel_softmax(ref.actor_targets(ns), un))
        probs = gumbel_softmax(ref.actors(st), uc)
        xmix = x.unsqueeze(0).repeat(K, 1, 1)
        for k in range(K):
            xmix[k, :, K * H * W + 9 * k: K * H * W + 9 * (k + 1)] = probs[k]
    checks = [(ref.actor_targets.net, ns.reshape(K, B, -1)), (ref.critic_targets, xt.unsqueeze(0).expand(K, -1, -1)),
              (ref.critics, x.unsqueeze(0).expand(K, -1, -1)), (ref.actors.net, st.reshape(K, B, -1)),
              (critic_after if critic_after is not None else ref.critics, xmix)]
    res = [_relu_margin(net, xi) for net, xi in checks]
    rows = torch.zeros(B, dtype=torch.bool, device=st.device)
    for _, r in res:
        rows |= r
    return rows, [m for m, _ in res]


def _grad_failures(got, want):
    """indices of the gradient tensors outside GRAD_TOL"""
    return [i for i, (a, b) in enumerate(zip(got, want)) if _rel(a, b) >= GRAD_TOL]


def _run_update(batch):
    """One update of a fresh (fused, autograd) pair on `batch`; the gradients and losses of both."""
    st, ac, rw, ns, dn, un, uc = batch
    ms = _pair()
    x = ms[1]._critic_in(st, ac).contiguous()
    xn = [ms[1]._critic_in(ns, torch.zeros_like(ac)).contiguous() for _ in range(2)]
    ctx = [m._learn_critic(st, ac, rw, ns, dn, un, (x.clone(), xn[i])) for i, m in enumerate(ms)]
    gc = (_grads(ms[0].critics), _grads(ms[1].critics))
    for i, m in enumerate(ms):
        m._learn_actor(ctx[i], uc)
    ga = (_grads(ms[0].actors.net), _grads(ms[1].actors.net))
    return ms, ctx, xn, gc, ga


def test_fused_gradients_match_autograd():
    g = torch.Generator(device="cuda").manual_seed(7)
    batch = list(_batch(g))
    st, ac, rw, ns, dn, un, uc = batch
    # every ReLU input the update evaluates (autograd's networks, float64): rows with one within
    # EDGE of zero could flip between the two summation orders -- mask them (a copy of a clean row;
    # the critic's Adam step depends on every row, so the check repeats after a mask) and require
    # that they are few
    masked = []
    for _ in range(4):
        ms, ctx, xn, gc, ga = _run_update(batch)
        st, ac, rw, ns, dn, un, uc = batch
        rows, margins = _edge_rows(_pair()[1], st, ac, ns, un, uc, critic_after=ms[1].critics)
        print("ReLU input margins per network:", margins, "edge rows:", rows.nonzero().flatten().tolist())
        if not rows.any():
            break
        clean = int((~rows).nonzero()[0])
        batch = [t.clone() for t in batch]
        st, ac, rw, ns, dn, un, uc = batch
        for b in rows.nonzero().flatten().tolist():
            masked.append(b)
            for t in (st, ac, ns, un, uc):
                t[:, b] = t[:, clean]
            rw[b], dn[b] = rw[clean], dn[clean]
    assert not rows.any() and len(masked) <= 3, masked
    D = K * H * W
    torch.testing.assert_close(xn[0][:, D:], xn[1][:, D:], rtol=0, atol=2e-6)       # target actions
    torch.testing.assert_close(ctx[0]["critic_loss"], ctx[1]["critic_loss"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(ctx[0]["actor_loss"], ctx[1]["actor_loss"], rtol=1e-4, atol=1e-6)
    print("critic grad rel L2:", ["%.1e" % _rel(a, b) for a, b in zip(*gc)])
    print("actor grad rel L2:", ["%.1e" % _rel(a, b) for a, b in zip(*ga)])
    assert not _grad_failures(*gc)
    assert not _grad_failures(*ga)
    # the bound bites: any single tensor perturbed by 1e-4 relative fails it
    for got, want in (gc, ga):
        for i in range(len(got)):
            bad = [t.clone() for t in got]
            bad[i] = bad[i] * (1.0 + 1e-4)
            assert _grad_failures(bad, want) == [i]


def test_fused_updates_match_per_agent_loop():
    from test_maddpg import PerAgentReference, _seq
    m = _pair()[0]
    ref = PerAgentReference(m, LR, LR)
    g = torch.Generator(device="cuda").manual_seed(1)
    steps = 4
    for it in range(steps):
        st, ac, rw, ns, dn, un, uc = _batch(g)
        a_loss, c_loss = m.learn(st, ac, rw, ns, dn, un, uc)
        want = ref.learn(st, ac, rw, ns, dn, un, uc)
        for k in range(K):
            assert abs(a_loss[k].item() - want[k][0]) < 1e-4 * max(1.0, abs(want[k][0]))
            assert abs(c_loss[k].item() - want[k][1]) < 1e-4 * max(1.0, abs(want[k][1]))
    # both step counts advanced once per update (by the gradient launches; the Adam launches read them)
    for opt in (m.opt_actor, m.opt_critic):
        assert opt.count.tolist() == [steps, 0]
    worst, rels = 0.0, []
    for k in range(K):
        for stacked, seqs in ((m.actors.net, ref.actors), (m.actor_targets.net, ref.actor_t),
                              (m.critics, ref.critics), (m.critic_targets, ref.critic_t)):
            for a, b in zip(_seq(stacked, k).parameters(), seqs[k].parameters()):
                rel = _rel(a.detach(), b.detach())
                worst = max(worst, rel)
                rels.append(rel)
                assert rel < 1e-5, rel
    print("worst parameter rel L2 after", steps, "updates:", worst)


def test_fused_graph_replay_equals_eager():
    ms = _pair()
    ms[1].fused = True
    g = torch.Generator(device="cuda").manual_seed(9)
    batch = _batch(g)
    ms[0].capture(batch=batch, warmup=2)
    for _ in range(2):
        ms[1].learn(*batch)
    for _ in range(3):
        ms[0].replay_learn()
        ms[1].learn(*batch)
    torch.cuda.synchronize()
    for a, b in zip(ms[0].state_dict().values(), ms[1].state_dict().values()):
        assert torch.equal(a, b)


@pytest.mark.parametrize("Bt,patch", [(32, 0), (128, 11)])
def test_fused_small_batch_and_patch_inputs(Bt, patch):
    """Other batch sizes and the local-window input (D = P * P): fused == autograd, same bound."""
    global H, W
    h0, w0 = H, W
    try:
        if patch:
            H = W = patch
        ms = [MADDPG(K, H, W, device="cuda", seed=5, batch_size=Bt) for _ in range(2)]
        ms[1].fused = False
        g = torch.Generator(device="cuda").manual_seed(3)
        st, ac, rw, ns, dn, un, uc = _batch(g, Bt)
        outs = [m.learn(st, ac, rw, ns, dn, un, uc) for m in ms]
        for a, b in zip(outs[0], outs[1]):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
        for a, b in zip(ms[0].state_dict().values(), ms[1].state_dict().values()):
            assert _rel(a, b) < 1e-5
    finally:
        H, W = h0, w0


def test_fused_learner_takes_any_batch_size():
    """the fused kernels take batches of 16-row tiles; a learner built with another
    batch size (agilerl accepts any, e.g. 100) runs the torch composition instead of raising, and
    its update equals the unfused learner's bit for bit (the same torch path)."""
    ms = _pair()
    g = torch.Generator(device="cuda").manual_seed(9)
    b = _batch(g, 100)
    for m in ms:
        m.learn(*b)
    for a, c in zip(ms[0].state_dict().values(), ms[1].state_dict().values()):
        assert torch.equal(a, c)
