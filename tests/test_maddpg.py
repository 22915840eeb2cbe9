"""The stacked GPU-shaped MADDPG update (marlnav/maddpg.py) == a plain per-agent PyTorch fp32
restatement of agilerl 1.0.15's MADDPG.learn loop (maddpg/agent.py:199-224 call site), agent by
agent: separate nn.Sequential actors/critics, separate Adam optimisers, critic step then actor
step per agent, soft target update at the end.  On the CPU the learner uses torch's Adam; the
GPU tests (marked gpu) run its HIP path (flat buffers, gw_adam_step, gw_soft_update) against
the same per-agent loop and against torch.optim.Adam; the graph-capture path is in
tests/test_gpu_rollout.py."""
import copy

import pytest
import torch
import torch.nn as nn

from marlnav.maddpg import MADDPG, gumbel_softmax, learns_per_step


def _seq(stacked, k, n_layers=3):
    """nn.Sequential copy of agent k of a StackedMLPActors (on the stacked net's device)."""
    dims = [stacked.weights[i].shape[1] for i in range(n_layers)] + [stacked.weights[-1].shape[2]]
    mods = []
    for i in range(n_layers):
        lin = nn.Linear(dims[i], dims[i + 1])
        with torch.no_grad():
            lin.weight.copy_(stacked.weights[i][k].t())
            lin.bias.copy_(stacked.biases[i][k, 0])
        mods.append(lin)
        if i < n_layers - 1:
            ln = nn.LayerNorm(dims[i + 1])
            with torch.no_grad():
                ln.weight.copy_(stacked.ln_w[i][k, 0])
                ln.bias.copy_(stacked.ln_b[i][k, 0])
            mods += [ln, nn.ReLU()]
    return nn.Sequential(*mods).to(stacked.weights[0].device)


class PerAgentReference:
    """agilerl-style MADDPG with one module and one Adam per agent and network."""

    def __init__(self, m: MADDPG, lr_a, lr_c):
        K = m.K
        self.K, self.gamma, self.tau = K, m.gamma, m.tau
        self.actors = [_seq(m.actors.net, k) for k in range(K)]
        self.actor_t = [_seq(m.actor_targets.net, k) for k in range(K)]
        self.critics = [_seq(m.critics, k) for k in range(K)]
        self.critic_t = [_seq(m.critic_targets, k) for k in range(K)]
        self.opt_a = [torch.optim.Adam(a.parameters(), lr=lr_a) for a in self.actors]
        self.opt_c = [torch.optim.Adam(c.parameters(), lr=lr_c) for c in self.critics]

    def learn(self, states, actions, rewards, next_states, dones, u_next, u_cur):
        K, B = states.shape[0], states.shape[1]
        s = [states[k].reshape(B, -1) for k in range(K)]
        ns = [next_states[k].reshape(B, -1) for k in range(K)]
        acts = [actions[k] for k in range(K)]
        with torch.no_grad():
            next_acts = [gumbel_softmax(self.actor_t[k](ns[k]), u_next[k]) for k in range(K)]
        x = torch.cat(s + acts, 1)
        x_next = torch.cat(ns + next_acts, 1)
        losses = []
        for k in range(K):
            q = self.critics[k](x)
            with torch.no_grad():
                q_next = self.critic_t[k](x_next)
            y = rewards[:, k:k + 1].float() + (1 - dones[:, k:k + 1].float()) * self.gamma * q_next
            closs = nn.MSELoss()(q, y)
            self.opt_c[k].zero_grad()
            closs.backward()
            self.opt_c[k].step()
            a_k = gumbel_softmax(self.actors[k](s[k]), u_cur[k])
            det = [a.detach() for a in acts]
            det[k] = a_k
            aloss = -self.critics[k](torch.cat(s + det, 1)).mean()
            self.opt_a[k].zero_grad()
            aloss.backward()
            self.opt_a[k].step()
            losses.append((aloss.item(), closs.item()))
        with torch.no_grad():
            for nets, tgts in ((self.actors, self.actor_t), (self.critics, self.critic_t)):
                for n, t in zip(nets, tgts):
                    for p, tp in zip(n.parameters(), t.parameters()):
                        tp.copy_(self.tau * p + (1 - self.tau) * tp)
        return losses


def _assert_same(m: MADDPG, ref: PerAgentReference, tol=2e-5):
    for k in range(m.K):
        for stacked, seqs in ((m.actors.net, ref.actors), (m.actor_targets.net, ref.actor_t),
                              (m.critics, ref.critics), (m.critic_targets, ref.critic_t)):
            want = _seq(stacked, k)
            for a, b in zip(want.parameters(), seqs[k].parameters()):
                torch.testing.assert_close(a, b, rtol=tol, atol=tol)


@pytest.mark.parametrize("K", [1, 2, 3])
def test_stacked_learn_matches_per_agent_loop(K):
    torch.manual_seed(0)
    H, W, B = 4, 5, 16
    m = MADDPG(K, H, W, hidden=(16, 16), lr_actor=1e-2, lr_critic=1e-2, gamma=0.98, tau=0.1, batch_size=B, seed=3)
    # make the targets differ from the online nets, as after some training
    with torch.no_grad():
        for p in list(m.actor_targets.parameters()) + list(m.critic_targets.parameters()):
            p.add_(0.05 * torch.randn_like(p))
    ref = PerAgentReference(m, 1e-2, 1e-2)
    g = torch.Generator().manual_seed(1)
    for it in range(4):
        states = torch.randint(-1, 6, (K, B, H, W), generator=g).float()
        next_states = torch.randint(-1, 6, (K, B, H, W), generator=g).float()
        actions = torch.softmax(torch.randn((K, B, 9), generator=g), -1)
        rewards = torch.randn((B, K), generator=g, dtype=torch.float64) * 10
        dones = (torch.rand((B, K), generator=g) < 0.2).to(torch.uint8)
        u_next = torch.rand((K, B, 9), generator=g)
        u_cur = torch.rand((K, B, 9), generator=g)
        a_loss, c_loss = m.learn(states, actions, rewards, next_states, dones, u_next, u_cur)
        want = ref.learn(states, actions, rewards, next_states, dones, u_next, u_cur)
        for k in range(K):
            assert abs(a_loss[k].item() - want[k][0]) < 1e-4 * max(1.0, abs(want[k][0]))
            assert abs(c_loss[k].item() - want[k][1]) < 1e-4 * max(1.0, abs(want[k][1]))
        _assert_same(m, ref)


@pytest.mark.gpu
def test_gpu_flat_learn_matches_per_agent_loop():
    """On the GPU the learner takes its HIP path (flat parameter buffers, gw_adam_step,
    gw_soft_update).  At the C3/C5 shape (32x32 obs, K = 2, batch 128, hidden 128-128, the
    configs/custom_fear_5.yaml learning rates) four updates == the per-agent fp32 loop with
    torch.optim.Adam on the same device.
    Tolerance: losses within 1e-4 relative; every parameter tensor within 1e-4 relative L2 error
    (GEMM summation order differs between the stacked bmm and the per-agent Linear, and Adam's
    normalised step turns rounding-level gradients into steps of up to lr, so elementwise
    bit-exactness is not expected) and within 2 * lr * steps elementwise."""
    torch.manual_seed(0)
    K, H, W, B, steps, lr = 2, 32, 32, 128, 4, 1e-3
    m = MADDPG(K, H, W, lr_actor=lr, lr_critic=lr, gamma=0.98, tau=0.01, batch_size=B, device="cuda", seed=3)
    assert m.flat  # the HIP optimizer / soft-update path
    m.fused = False  # the autograd composition (the fused kernels: tests/test_maddpg_fused.py)
    with torch.no_grad():
        for net in (m.actor_targets.net, m.critic_targets):
            net.flat_params().add_(0.05 * torch.randn_like(net.flat_params()))
    ref = PerAgentReference(m, lr, lr)
    g = torch.Generator(device="cuda").manual_seed(1)
    for it in range(steps):
        states = torch.randint(-1, 6, (K, B, H, W), generator=g, device="cuda").float()
        next_states = torch.randint(-1, 6, (K, B, H, W), generator=g, device="cuda").float()
        actions = torch.softmax(torch.randn((K, B, 9), generator=g, device="cuda"), -1)
        rewards = torch.randn((B, K), generator=g, dtype=torch.float64, device="cuda") * 10
        dones = (torch.rand((B, K), generator=g, device="cuda") < 0.2).to(torch.uint8)
        u_next = torch.rand((K, B, 9), generator=g, device="cuda")
        u_cur = torch.rand((K, B, 9), generator=g, device="cuda")
        a_loss, c_loss = m.learn(states, actions, rewards, next_states, dones, u_next, u_cur)
        want = ref.learn(states, actions, rewards, next_states, dones, u_next, u_cur)
        for k in range(K):
            assert abs(a_loss[k].item() - want[k][0]) < 1e-4 * max(1.0, abs(want[k][0]))
            assert abs(c_loss[k].item() - want[k][1]) < 1e-4 * max(1.0, abs(want[k][1]))
    for k in range(K):
        for stacked, seqs in ((m.actors.net, ref.actors), (m.actor_targets.net, ref.actor_t),
                              (m.critics, ref.critics), (m.critic_targets, ref.critic_t)):
            for a, b in zip(_seq(stacked, k).parameters(), seqs[k].parameters()):
                rel = float((a - b).norm() / b.norm().clamp_min(1e-12))
                assert rel < 1e-4, rel
                assert float((a - b).abs().max()) <= 2 * lr * steps


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 300_001])
def test_gpu_adam_and_soft_update_match_torch(n):
    """gw_adam_step == torch.optim.Adam (single-tensor, non-capturable) over 6 steps on the same
    flat buffer and gradients; gw_soft_update == tau * p + (1 - tau) * t in torch f32 (bit for
    bit) and p.lerp_ within 2 ulp-scale tolerance."""
    from marlnav import _lib
    from marlnav.actor import StackedMLPActors
    from marlnav.maddpg import FlatAdam
    torch.manual_seed(1)
    net = StackedMLPActors(1, 4, (4, 4), device="cuda")  # a FlatAdam host; its buffer is swapped below
    flat = torch.nn.Parameter(torch.randn(n, device="cuda"))
    flat.grad = torch.zeros_like(flat)
    net.flat_params = lambda: flat
    opt = FlatAdam(net, lr=1e-3)
    ref = torch.nn.Parameter(flat.detach().clone())
    topt = torch.optim.Adam([ref], lr=1e-3, foreach=False, capturable=False)
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(6):
        grad = torch.randn(n, device="cuda", generator=g) * torch.rand(n, device="cuda", generator=g) * 3
        flat.grad.copy_(grad)
        ref.grad = grad.clone()
        opt.step()
        topt.step()
        torch.testing.assert_close(flat.detach(), ref.detach(), rtol=2e-6, atol=1e-7)
        # the same ops and roundings as torch's single-tensor Adam (fmas where torch's contracted
        # elementwise kernels fuse); tolerance: a few f32 ulps of the moment's scale, since a
        # contraction difference inside lerp / addcmul shows up where the moment nearly cancels
        for mine, theirs in ((opt.m, topt.state[ref]["exp_avg"]), (opt.v, topt.state[ref]["exp_avg_sq"])):
            scale = float(theirs.abs().max())
            torch.testing.assert_close(mine, theirs, rtol=1e-6, atol=4e-7 * scale)
    assert int(opt.count[0]) == 6 and int(opt.count[1]) == 0
    lib = _lib.load()
    t = torch.randn(n, device="cuda")
    p = torch.randn(n, device="cuda")
    want = 0.01 * p + (1.0 - 0.01) * t
    lerp = t.clone().lerp_(p, 0.01)
    _lib.check(lib.gw_soft_update(t.data_ptr(), p.data_ptr(), n, 0.01,
                                  torch.cuda.current_stream().cuda_stream), "gw_soft_update")
    torch.testing.assert_close(t, want, rtol=2e-7, atol=1e-7)
    torch.testing.assert_close(t, lerp, rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("n,n2", [(1000, 3000), (300_001, 77)])
def test_gpu_adam_soft_step_equals_adam_then_soft_update(n, n2):
    """gw_adam_soft_step (the learner's last launch) == gw_adam_step followed by gw_soft_update2,
    bit for bit: parameters, moments, step count and both targets, over 3 steps.  The soft step
    runs with advanced = 1 (its count advanced beforehand, as the fused gradient launch does), the
    plain step advances its own count (the arrival counter)."""
    from marlnav import _lib
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(4)
    bufs = []
    for _ in range(2):
        torch.manual_seed(9)
        bufs.append(dict(p=torch.randn(n, device="cuda"), m=torch.zeros(n, device="cuda"), v=torch.zeros(n, device="cuda"),
                         c=torch.zeros(2, dtype=torch.int32, device="cuda"), t1=torch.randn(n, device="cuda"),
                         t2=torch.randn(n2, device="cuda"), o2=torch.randn(n2, device="cuda")))
    for _ in range(3):
        grad = torch.randn(n, device="cuda", generator=g)
        a, b = bufs
        _lib.check(lib.gw_adam_step(a["p"].data_ptr(), grad.data_ptr(), a["m"].data_ptr(), a["v"].data_ptr(),
                                    a["c"].data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8, 0, s), "gw_adam_step")
        _lib.check(lib.gw_soft_update2(a["t1"].data_ptr(), a["p"].data_ptr(), n, a["t2"].data_ptr(), a["o2"].data_ptr(),
                                       n2, 0.01, s), "gw_soft_update2")
        b["c"][0] += 1  # the count advanced by a preceding launch
        _lib.check(lib.gw_adam_soft_step(b["p"].data_ptr(), grad.data_ptr(), b["m"].data_ptr(), b["v"].data_ptr(),
                                         b["c"].data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8, b["t1"].data_ptr(), 0.01,
                                         b["t2"].data_ptr(), b["o2"].data_ptr(), n2, 1, s), "gw_adam_soft_step")
    torch.cuda.synchronize()
    for key in ("p", "m", "v", "c", "t1", "t2"):
        assert torch.equal(bufs[0][key], bufs[1][key]), key
    assert int(bufs[1]["c"][0]) == 3 and int(bufs[1]["c"][1]) == 0


def test_gumbel_softmax_is_a_distribution_and_sharpens():
    logits = torch.tensor([[0.0, 5.0, 0.0]])
    g = torch.Generator().manual_seed(0)
    p = torch.stack([gumbel_softmax(logits, generator=g) for _ in range(2000)])
    torch.testing.assert_close(p.sum(-1), torch.ones_like(p.sum(-1)))
    assert (p.argmax(-1) == 1).float().mean() > 0.9


def test_learn_schedule_matches_reference_rule():
    # maddpg/agent.py:199-224: learn_step > num_envs -> every learn_step // num_envs steps
    assert [learns_per_step(1, 10, i) for i in range(21)].count(1) == 3
    assert learns_per_step(4, 10, 0) == 1 and learns_per_step(4, 10, 1) == 0
    # num_envs >= learn_step -> num_envs // learn_step learns every step
    assert learns_per_step(65536, 10, 7) == 6553


def test_checkpoint_roundtrip(tmp_path):
    m = MADDPG(2, 4, 5, hidden=(8, 8), seed=1)
    path = str(tmp_path / "maddpg.safetensors")
    m.save(path)
    m2 = MADDPG(2, 4, 5, hidden=(8, 8), seed=7)
    m2.load(path)
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)
    m3 = copy.deepcopy(m2)
    assert torch.equal(m3.actors.net.weights[0], m.actors.net.weights[0])


@pytest.mark.gpu
def test_gpu_learn_from_critic_rows_equals_assembled():
    """ReplayRing.sample(critic_in=True) returns the critic's input rows that MADDPG.learn would
    assemble (agent-major states + the stored action probabilities) bit for bit, and learning
    from them (target actions written into x_next's slots by gw_gumbel_softmax) leaves every
    network bit-identical to the assembling path."""
    from marlnav.rollout import Rollout
    from marlnav.vec_env import VecGridEnv
    env = VecGridEnv("grid32", num_envs=256, fear=True, fear_weight=-5.0, seed=1, stats=True, final_obs=True)
    ms = [MADDPG(env.K, env.H, env.W, device="cuda", seed=1) for _ in range(2)]
    ro = Rollout(env, ms[0].actors, replay_slots=8, training=True, seed=2)
    ro.reset()
    for _ in range(12):
        ro.step()
    ro.fence()
    for it in range(3):
        g = torch.Generator(device="cuda").manual_seed(10 + it)
        *batch, (x, xn) = ro.replay.sample(64, generator=g, critic_in=True)
        states, actions, rewards, next_states, dones = batch
        assert torch.equal(x, ms[1]._critic_in(states, actions))
        D = env.K * env.H * env.W
        assert torch.equal(xn[:, :D], next_states.reshape(env.K, 64, -1).permute(1, 0, 2).reshape(64, -1))
        u_next = torch.rand((env.K, 64, 9), device="cuda", generator=g)
        u_cur = torch.rand((env.K, 64, 9), device="cuda", generator=g)
        la = ms[0].learn(*batch, u_next=u_next, u_cur=u_cur, critic_in=(x, xn))
        lb = ms[1].learn(*batch, u_next=u_next, u_cur=u_cur)
        assert torch.equal(la[0], lb[0]) and torch.equal(la[1], lb[1])
    for a, b in ((ms[0].actors.net, ms[1].actors.net), (ms[0].critics, ms[1].critics),
                 (ms[0].actor_targets.net, ms[1].actor_targets.net), (ms[0].critic_targets, ms[1].critic_targets)):
        assert torch.equal(a.flat_params(), b.flat_params())
    env.close()


@pytest.mark.gpu
def test_gpu_td_target_and_paired_soft_update_bit_exact():
    """gw_td_target == torch's r + (1 - d) * gamma * q_next (f64 reward and u8 done converted to
    f32 first) bit for bit; gw_soft_update2 == two gw_soft_update launches bit for bit."""
    from marlnav import _lib
    K, B = 2, 128
    m = MADDPG(K, 4, 4, device="cuda", seed=0)
    g = torch.Generator(device="cuda").manual_seed(3)
    rewards = torch.randn((B, K), generator=g, dtype=torch.float64, device="cuda") * 37
    dones = (torch.rand((B, K), generator=g, device="cuda") < 0.3).to(torch.uint8)
    q_next = torch.randn((K, B, 1), generator=g, device="cuda") * 11
    want = rewards.to(torch.float32).t().unsqueeze(-1) + (1.0 - dones.to(torch.float32).t().unsqueeze(-1)) * m.gamma * q_next
    assert torch.equal(m._td_target(rewards, dones, q_next), want)
    lib, s = _lib.load(), torch.cuda.current_stream().cuda_stream
    t1, p1 = torch.randn(1001, device="cuda", generator=g), torch.randn(1001, device="cuda", generator=g)
    t2, p2 = torch.randn(70_000, device="cuda", generator=g), torch.randn(70_000, device="cuda", generator=g)
    a1, a2 = t1.clone(), t2.clone()
    _lib.check(lib.gw_soft_update(a1.data_ptr(), p1.data_ptr(), 1001, 0.01, s), "gw_soft_update")
    _lib.check(lib.gw_soft_update(a2.data_ptr(), p2.data_ptr(), 70_000, 0.01, s), "gw_soft_update")
    _lib.check(lib.gw_soft_update2(t1.data_ptr(), p1.data_ptr(), 1001, t2.data_ptr(), p2.data_ptr(), 70_000, 0.01, s),
               "gw_soft_update2")
    assert torch.equal(t1, a1) and torch.equal(t2, a2)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [128, 100])
def test_gpu_mean_losses_match_torch(B):
    """gw_mean_loss_fwd / _bwd (the critic's MSELoss and the actor's -mean Q per agent): the
    gradient equals torch's bit for bit; the loss values (another summation order) within 1e-6
    relative."""
    from marlnav.maddpg import _MeanLoss
    g = torch.Generator(device="cuda").manual_seed(B)
    q0 = torch.randn((3, B, 1), generator=g, device="cuda") * 5
    y = torch.randn((3, B, 1), generator=g, device="cuda") * 5
    for mode in (0, 1):
        qa, qb = q0.clone().requires_grad_(True), q0.clone().requires_grad_(True)
        la = _MeanLoss.apply(qa, y if mode == 0 else None, mode)
        lb = ((qb - y) ** 2).mean(dim=(1, 2)) if mode == 0 else -qb.mean(dim=(1, 2))
        torch.testing.assert_close(la, lb, rtol=1e-6, atol=1e-6)
        la.sum().backward()
        lb.sum().backward()
        assert torch.equal(qa.grad, qb.grad)


def _split_vs_concat(device):
    K, H, W, B = 2, 32, 32, 128
    m = MADDPG(K, H, W, device=device, seed=4)
    g = torch.Generator(device=device).manual_seed(5)
    states = torch.randint(-1, 14, (K, B, H, W), generator=g, device=device).float()
    actions = torch.softmax(torch.randn((K, B, 9), generator=g, device=device) * 3, -1)
    x = m._critic_in(states, actions)
    with torch.no_grad():
        q_cat = m.critics(x.unsqueeze(0).expand(K, -1, -1))
        a_rep = x[:, K * H * W:].unsqueeze(0).expand(K, -1, -1).contiguous()
        q_split = m._q_split(x, a_rep)
    return q_cat, q_split


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_split_q_matches_concat_q(device):
    """The actor loss evaluates the critic with layer 1 split into state and action columns
    (MADDPG._q_split); on rows whose action slots hold the replayed actions that is the critic's
    forward on the concatenated input (agilerl's single Linear over torch.cat) up to f32
    summation order.  Tolerance: 2e-5 relative + 2e-5 absolute on Q (a 2,066-term f32 dot product
    split in two partial sums; layer-2/3 LayerNorms keep the scale ~1)."""
    q_cat, q_split = _split_vs_concat(device)
    torch.testing.assert_close(q_split, q_cat, rtol=2e-5, atol=2e-5)


@pytest.mark.gpu
def test_gpu_capture_without_warmup_then_eager_learn():
    """MADDPG.capture(warmup=0) records the update without running it; an eager learn before the
    first replay must equal a twin that never captured (bit for bit): nothing the capture records
    (e.g. a cached ones tensor for the bias gradients) may be read before it is filled."""
    from marlnav.actor import _StackedLinear
    from marlnav.rollout import Rollout
    from marlnav.vec_env import VecGridEnv
    _StackedLinear._ones.clear()
    env = VecGridEnv("grid32", num_envs=256, fear=True, fear_weight=-5.0, seed=1, stats=True, final_obs=True)
    ms = [MADDPG(env.K, env.H, env.W, device="cuda", seed=1, capturable=True) for _ in range(2)]
    ro = Rollout(env, ms[0].actors, replay_slots=8, training=True, seed=2)
    ro.reset()
    for _ in range(6):
        ro.step()
    ro.fence()
    ms[0].capture(ro.replay, warmup=0)
    torch.cuda.manual_seed(7)  # the Gumbel uniforms come from the default generator
    ms[0].learn_from(ro.replay, generator=torch.Generator(device="cuda").manual_seed(3))
    _StackedLinear._ones.clear()  # the twin builds its own cache eagerly
    torch.cuda.manual_seed(7)
    ms[1].learn_from(ro.replay, generator=torch.Generator(device="cuda").manual_seed(3))
    torch.cuda.synchronize()
    for a, b in ((ms[0].actors.net, ms[1].actors.net), (ms[0].critics, ms[1].critics)):
        assert torch.equal(a.flat_params(), b.flat_params())
    env.close()


def test_checkpoint_keeps_optimizer_state(tmp_path):
    """MADDPG.save / load carry the optimizers (agilerl's save_checkpoint keeps them): a restored
    learner's next update equals the original's (CPU, torch Adam state per parameter)."""
    K, H, W, B = 2, 4, 5, 8
    m = MADDPG(K, H, W, hidden=(8, 8), batch_size=B, seed=1)
    g = torch.Generator().manual_seed(0)

    def batch():
        return (torch.randint(-1, 6, (K, B, H, W), generator=g).float(), torch.softmax(torch.randn((K, B, 9), generator=g), -1),
                torch.randn((B, K), generator=g, dtype=torch.float64), torch.randint(-1, 6, (K, B, H, W), generator=g).float(),
                (torch.rand((B, K), generator=g) < 0.2).to(torch.uint8), torch.rand((K, B, 9), generator=g),
                torch.rand((K, B, 9), generator=g))
    for _ in range(3):
        m.learn(*batch())
    path = str(tmp_path / "ck.safetensors")
    m.save(path)
    m2 = MADDPG(K, H, W, hidden=(8, 8), batch_size=B, seed=9)
    m2.load(path)
    b = batch()
    m.learn(*b)
    m2.learn(*b)
    for a, c in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, c)


def test_cnn_optimizer_load_is_in_place_cpu():
    """loading the optimizer state must write into the existing Adam state tensors
    (a captured update graph with capturable Adam keeps reading and writing those very tensors),
    not replace them.  CNN arch (per-parameter torch Adam), CPU: the state tensors keep their
    storage and take the loaded values."""
    K, H, W, B = 2, 8, 8, 4
    m = MADDPG(K, H, W, arch="cnn", batch_size=B, seed=1)
    g = torch.Generator().manual_seed(0)

    def batch():
        return (torch.randint(-1, 6, (K, B, H, W), generator=g).float(), torch.softmax(torch.randn((K, B, 9), generator=g), -1),
                torch.randn((B, K), generator=g, dtype=torch.float64), torch.randint(-1, 6, (K, B, H, W), generator=g).float(),
                (torch.rand((B, K), generator=g) < 0.2).to(torch.uint8), torch.rand((K, B, 9), generator=g),
                torch.rand((K, B, 9), generator=g))
    m.learn(*batch())
    sd = {k: v.clone() + 1.0 for k, v in m.optim_state_dict().items()}
    ptrs = {id(p): {k: t.data_ptr() for k, t in st.items()} for opt in (m.opt_actor, m.opt_critic)
            for p, st in opt.state.items()}
    m.load_optim_state_dict(sd)
    for name, opt in (("opt_actor", m.opt_actor), ("opt_critic", m.opt_critic)):
        for i, p in enumerate(opt.param_groups[0]["params"]):
            st = opt.state[p]
            for key in ("exp_avg", "exp_avg_sq", "step"):
                assert st[key].data_ptr() == ptrs[id(p)][key]
                assert torch.equal(st[key], sd[f"{name}.{i}.{key}"].to(st[key].dtype))
