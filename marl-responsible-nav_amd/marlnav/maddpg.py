"""MADDPG learner on the GPU: agilerl 1.0.15 ``MADDPG.learn`` restated for K stacked agents, with the
whole update (replay sampling, target actions, critic and actor steps, soft target update)
capturable as one HIP graph.

Reference call sites: ``maddpg/agent.py:41-65`` (construction from ``configs/custom_fear_5.yaml``:
LR_ACTOR = LR_CRITIC = 1e-3, GAMMA = 0.98, TAU = 0.01, BATCH_SIZE = 128, LEARN_STEP = 10,
MEMORY_SIZE = 200000), ``:199-224`` (sample + learn schedule) and ``:190-197`` (what is stored:
state, the GumbelSoftmax action probabilities, shaped reward, next_state, termination).

agilerl is not installed, so its published algorithm is restated here ("parity
unpinned" for its stochastic parts; tests/test_maddpg.py checks this batched form against a
plain per-agent PyTorch fp32 restatement of the same update, agent by agent):

  x  = [s_1 .. s_K, a_1 .. a_K]                      (flattened obs, action probabilities)
  a'_k = GumbelSoftmax(actor_target_k(s'_k))         (detached)
  y_k  = r_k + (1 - d_k) * gamma * critic_target_k([s'_1 .. s'_K, a'_1 .. a'_K])
  critic_k  <- Adam step on  MSE(critic_k(x), y_k)
  actor_k   <- Adam step on  -mean(critic_k(x with a_k := GumbelSoftmax(actor_k(s_k))))
               (after the critic step; the other agents keep their replayed actions)
  targets   <- tau * online + (1 - tau) * target      (after all agents)

The K agents' parameters are disjoint and every agent's losses only read replayed data and
detached target actions, so running the K updates together (stacked [K, ...] weights, one
batched GEMM chain, the K losses summed before one backward, one Adam over the stacked
tensors) is the same arithmetic as agilerl's per-agent loop.  Critic: the MLP of the shipped
checkpoints' critic layout (input K*H*W + K*9 -> 128 -> 128 -> 1, LayerNorm, ReLU).
"""
from __future__ import annotations

import copy

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import _lib
from .actor import N_ACTIONS, MultiAgentActors, StackedMLPActors


class _MeanLoss(torch.autograd.Function):
    """Per-agent loss over q [K, B, 1]: MSE against y (mode 0) or -mean q (mode 1), forward and
    backward one launch each (gw_mean_loss_fwd / _bwd); the gradient is torch's bit for bit."""

    @staticmethod
    def forward(ctx, q, y, mode):
        K, B = q.shape[0], q.shape[1]
        q = q.contiguous()
        y = y.contiguous() if y is not None else None
        loss = torch.empty((K,), device=q.device, dtype=q.dtype)
        _lib.check(_lib.load().gw_mean_loss_fwd(q.data_ptr(), y.data_ptr() if y is not None else None, loss.data_ptr(),
                                                K, B, mode, torch.cuda.current_stream(q.device).cuda_stream),
                   "gw_mean_loss_fwd")
        ctx.save_for_backward(q, y) if y is not None else ctx.save_for_backward(q)
        ctx.mode = mode
        return loss

    @staticmethod
    def backward(ctx, g):
        saved = ctx.saved_tensors
        q, y = saved[0], (saved[1] if len(saved) > 1 else None)
        K, B = q.shape[0], q.shape[1]
        dq = torch.empty_like(q)
        _lib.check(_lib.load().gw_mean_loss_bwd(q.data_ptr(), y.data_ptr() if y is not None else None,
                                                g.contiguous().data_ptr(), dq.data_ptr(), K, B, ctx.mode,
                                                torch.cuda.current_stream(q.device).cuda_stream), "gw_mean_loss_bwd")
        return dq, None, None


def _gumbel_into_slots(logits: torch.Tensor, u: torch.Tensor | None, x_next: torch.Tensor, D: int):
    """GumbelSoftmax of the target logits [K, B, 9] written straight into the action slots
    x_next[:, D:] of the critic's input rows [B, D + K*9] (gw_gumbel_softmax, strided output)."""
    K, B, n = logits.shape
    if not (x_next.is_cuda and x_next.dtype == torch.float32 and x_next.is_contiguous()
            and tuple(x_next.shape) == (B, D + K * n) and x_next.device == logits.device):
        raise ValueError(f"critic input rows must be a contiguous float32 [B, D + K*9] = [{B}, {D + K * n}] CUDA "
                         f"tensor on the logits' device, got {tuple(x_next.shape)} {x_next.dtype}")
    logits = logits.contiguous()
    if u is None:
        u = torch.rand(logits.shape, device=logits.device, dtype=logits.dtype)
    if tuple(u.shape) != (K, B, n) or u.dtype != torch.float32:
        raise ValueError("u must be float32 [K, B, 9]")
    u = u.contiguous()
    _lib.check(_lib.load().gw_gumbel_softmax(logits.data_ptr(), u.data_ptr(), x_next[:, D:].data_ptr(), K * B, n, 1.0,
                                             1e-20, B, x_next.shape[1],
                                             torch.cuda.current_stream(logits.device).cuda_stream), "gw_gumbel_softmax")


def _gumbel_hip(logits: torch.Tensor, u: torch.Tensor | None, tau: float = 1.0, eps: float = 1e-20) -> torch.Tensor:
    """The learner's target actions: gumbel_softmax as ONE gw_gumbel_softmax
    launch (no gradient).  Its sum order and logf / expf differ from the torch formula by ~2e-6
    relative, so the public ``gumbel_softmax`` stays the torch formula (the tests' reference)."""
    logits = logits.contiguous()
    if u is None:
        u = torch.rand(logits.shape, device=logits.device, dtype=logits.dtype)
    u = u.contiguous()
    out = torch.empty_like(logits)
    n = logits.shape[-1]
    _lib.check(_lib.load().gw_gumbel_softmax(logits.data_ptr(), u.data_ptr(), out.data_ptr(), logits.numel() // n,
                                             n, tau, eps, 0, 0, torch.cuda.current_stream(logits.device).cuda_stream),
               "gw_gumbel_softmax")
    return out


def gumbel_softmax(logits: torch.Tensor, u: torch.Tensor | None = None, tau: float = 1.0, eps: float = 1e-20,
                   generator: torch.Generator | None = None) -> torch.Tensor:
    """agilerl's GumbelSoftmax output activation: softmax((logits - log(-log(u + eps) + eps)) / tau)
    (plain torch ops)."""
    if u is None:
        u = torch.rand(logits.shape, device=logits.device, dtype=logits.dtype, generator=generator)
    return F.softmax((logits - torch.log(-torch.log(u + eps) + eps)) / tau, dim=-1)


class FlatAdam:
    """torch.optim.Adam semantics over one StackedMLPActors' flat parameter buffer with the
    hand-written gw_adam_step kernel (include/learner_ops.h): one grid-stride launch per step,
    the step count on the device (graph-capturable)."""

    def __init__(self, net: StackedMLPActors, lr: float, betas=(0.9, 0.999), eps: float = 1e-8):
        self.net = net
        self.flat = net.flat_params()
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        # [0] steps taken, [1] the Adam launch's arrival counter (gw_adam_step; stays 0 between steps)
        self.count = torch.zeros(2, dtype=torch.int32, device=self.flat.device)
        self.lr, self.betas, self.eps = float(lr), betas, float(eps)
        self.lib = _lib.load()

    def zero_grad(self, set_to_none: bool = False):
        self.flat.grad.zero_()  # the per-layer .grad views accumulate into this buffer

    def step(self, advanced: bool = False):
        """advanced: the preceding gradient launch already advanced the step count (the fused
        learner's gw_maddpg_*_grads(adam_step=count)), so the Adam launch only reads it."""
        s = torch.cuda.current_stream(self.flat.device).cuda_stream
        _lib.check(self.lib.gw_adam_step(self.flat.data_ptr(), self.flat.grad.data_ptr(), self.m.data_ptr(),
                                         self.v.data_ptr(), self.count.data_ptr(), self.flat.numel(), self.lr,
                                         self.betas[0], self.betas[1], self.eps, int(advanced), s), "gw_adam_step")
        self.net.epoch += 1  # written behind torch's version counter (see MultiAgentActors.act_env)

    def step_soft(self, target: torch.Tensor, tau: float, target2: torch.Tensor, online2: torch.Tensor,
                  advanced: bool = False):
        """step(), then the soft target updates target <- tau p + (1 - tau) target (this buffer's
        target) and target2 <- tau online2 + (1 - tau) target2, in ONE launch (gw_adam_soft_step)."""
        s = torch.cuda.current_stream(self.flat.device).cuda_stream
        _lib.check(self.lib.gw_adam_soft_step(self.flat.data_ptr(), self.flat.grad.data_ptr(), self.m.data_ptr(),
                                              self.v.data_ptr(), self.count.data_ptr(), self.flat.numel(), self.lr,
                                              self.betas[0], self.betas[1], self.eps, target.data_ptr(), float(tau),
                                              target2.data_ptr(), online2.data_ptr(), online2.numel(),
                                              int(advanced), s),
                   "gw_adam_soft_step")
        self.net.epoch += 1


def _mlp_target(net: StackedMLPActors) -> StackedMLPActors:
    """A frozen copy with its own flat buffer (copy.deepcopy would clone the layer views apart)."""
    K, in_dim = net.K, net.in_dim
    hidden = tuple(w.shape[2] for w in net.weights[:-1])
    t = StackedMLPActors(K, in_dim, hidden, n_actions=net.weights[-1].shape[2], layer_norm=net.layer_norm,
                         device=net.flat_params().device, dtype=net.flat_params().dtype)
    with torch.no_grad():
        t.flat_params().copy_(net.flat_params())
    t.requires_grad_(False)
    return t


def _mlp_spec(net: StackedMLPActors, grad: bool = False):
    """gw_mlp_actors of a StackedMLPActors (in -> 128 -> LN -> 128 -> LN -> out): its parameters,
    or (grad=True) their .grad views in the flat gradient buffer."""
    f = (lambda t: t.grad) if grad else (lambda t: t)
    ts = (net.weights[0], net.biases[0], net.ln_w[0], net.ln_b[0], net.weights[1], net.biases[1],
          net.ln_w[1], net.ln_b[1], net.weights[2], net.biases[2])
    return _lib.GwMlpActors(net.K, net.in_dim, 128, net.weights[2].shape[2], 1, *[f(t).data_ptr() for t in ts])


def _fusable_net(net: StackedMLPActors) -> bool:
    return (net.n_layers == 3 and net.layer_norm and net.weights[0].shape[2] == 128
            and tuple(net.weights[1].shape[1:]) == (128, 128) and net.flat_params().dtype == torch.float32)


class MADDPG:
    """K MADDPG agents with stacked networks.  ``actors`` is a MultiAgentActors (mlp or cnn).

    Data-parallel across ranks when a torch.distributed group of more
    than one rank exists (``group``, default the world): the networks are broadcast from rank 0
    at construction (``broadcast_parameters``), every rank learns on its own sampled batch, and
    each of the two backward passes is followed by ONE all-reduce of that network's flat gradient
    buffer, averaged over the ranks, before its Adam step, so the replicas stay identical.  Equal
    per-rank batches make the averaged gradient that of the mean loss over the concatenated
    batch (tests/test_maddpg_dp.py)."""

    def __init__(self, K: int, H: int, W: int, arch: str = "mlp", hidden=(128, 128), lr_actor: float = 1e-3,
                 lr_critic: float = 1e-3, gamma: float = 0.98, tau: float = 0.01, batch_size: int = 128,
                 learn_step: int = 10, device=None, seed: int = 0, capturable: bool = False, group=None):
        self.K, self.H, self.W, self.arch = K, H, W, arch
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.gamma, self.tau, self.batch_size, self.learn_step = gamma, tau, batch_size, learn_step
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.actors = MultiAgentActors(K, H, W, arch, hidden, device=self.device, seed=seed)
        self.critics = StackedMLPActors(K, K * H * W + K * N_ACTIONS, hidden, n_actions=1, device=self.device,
                                        seed=seed + 1)
        # on the GPU with MLP actors every network is one flat buffer: flat Adam + one-launch soft
        # updates (learner_ops.hip); otherwise (CPU, CNN actors) torch's Adam and foreach ops
        self.flat = self.device.type == "cuda" and arch == "mlp"
        if self.flat:
            self.actor_targets = copy.deepcopy(self.actors)
            self.actor_targets.net = _mlp_target(self.actors.net)
            self.critic_targets = _mlp_target(self.critics)
            self.opt_actor = FlatAdam(self.actors.net, lr_actor)
            self.opt_critic = FlatAdam(self.critics, lr_critic)
        else:
            # MLP targets with their own flat buffer (every layer a view of it, like the online
            # nets; copy.deepcopy would clone the layer views apart from it)
            self.actor_targets = copy.deepcopy(self.actors)
            if arch == "mlp":
                self.actor_targets.net = _mlp_target(self.actors.net)
            self.critic_targets = _mlp_target(self.critics)
            opt = dict(capturable=True) if capturable and self.device.type == "cuda" else {}
            self.opt_actor = torch.optim.Adam(self.actors.parameters(), lr=lr_actor, **opt)
            self.opt_critic = torch.optim.Adam(self.critics.parameters(), lr=lr_critic, **opt)
        for m in (self.actor_targets, self.critic_targets):
            m.requires_grad_(False)
        self._graph = None
        self._graphs = None  # world > 1: three graph segments between the gradient all-reduces
        # the fused update (csrc/maddpg_ops.hip: two launch sequences carry the two backward
        # passes; GW_FUSED_LEARN=0 selects the torch-autograd composition)
        import os
        self.fused = (self.flat and os.environ.get("GW_FUSED_LEARN", "1") != "0"
                      and all(_fusable_net(n) for n in (self.actors.net, self.actor_targets.net, self.critics,
                                                       self.critic_targets)))
        self._fws = {}
        self._desc = {}           # the descriptor learner's per-ring state (workspace, ABI structs)
        self._desc_stale = True   # its c1 partial sums need gw_maddpg_desc_prime before the next update
        # the key of the fused update's in-kernel draws (replay sample rows, Gumbel uniforms):
        # Philox(key; row, the critic optimizer's step count, tag), one key per rank (each rank
        # samples its own batch); the step count makes every update's draws new
        rank = dist.get_rank(group) if self.world > 1 else 0
        self._draw_key = (int(seed) * 0x9E3779B97F4A7C15 + 7919 * rank + 1) & 0xFFFFFFFFFFFFFFFF
        if self.world > 1:
            self.broadcast_parameters()

    # ---------------------------------------------------------------------------------------
    def _networks(self):
        """(name, module, flat parameter buffer or None) of the four networks."""
        mlp = self.arch == "mlp"
        return (("actor", self.actors, self.actors.net.flat_params() if mlp else None),
                ("actor_target", self.actor_targets, self.actor_targets.net.flat_params() if mlp else None),
                ("critic", self.critics, self.critics.flat_params()),
                ("critic_target", self.critic_targets, self.critic_targets.flat_params()))

    @torch.no_grad()
    def broadcast_parameters(self, src: int = 0):
        """Every network's parameters from rank ``src`` (one broadcast per flat buffer; the CNN
        actors' parameters coalesced into one), so all replicas act and learn identically."""
        if self.world <= 1:
            return
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        for _, module, flat in self._networks():
            if flat is not None:
                dist.broadcast(flat.detach(), src, group=self.group)
                continue
            ps = [p.detach() for p in module.parameters()]
            buf = _flatten_dense_tensors(ps)
            dist.broadcast(buf, src, group=self.group)
            for p, v in zip(ps, _unflatten_dense_tensors(buf, ps)):
                p.copy_(v)
        self.actors.mark_updated()
        self.actor_targets.mark_updated()
        for m in (self.critics, self.critic_targets):
            m.epoch += 1
        self._desc_stale = True

    @torch.no_grad()
    def _allreduce_grads(self, which: str):
        """Average ``which`` ("actor" / "critic") gradients over the ranks: one all-reduce of the
        network's flat gradient buffer (MLP), or of its coalesced gradients (CNN actors)."""
        if self.world <= 1:
            return
        module = self.critics if which == "critic" else self.actors
        if which == "critic" or self.arch == "mlp":
            g = (module if which == "critic" else module.net).flat_params().grad
            dist.all_reduce(g, group=self.group)
            g.mul_(1.0 / self.world)
            return
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        gs = [p.grad for p in module.parameters() if p.grad is not None]
        buf = _flatten_dense_tensors(gs)
        dist.all_reduce(buf, group=self.group)
        buf.mul_(1.0 / self.world)
        for g, v in zip(gs, _unflatten_dense_tensors(buf, gs)):
            g.copy_(v)

    # ---------------------------------------------------------------------------------------
    def _critic_in(self, states: torch.Tensor, actions: torch.Tensor) -> torch.Tensor:
        """[K, B, H, W] obs + [K, B, 9] actions -> [B, K*H*W + K*9] (agent-major, as agilerl's
        torch.cat(list(states.values()) + actions, 1))."""
        K, B = states.shape[0], states.shape[1]
        s = states.reshape(K, B, -1).permute(1, 0, 2).reshape(B, -1)
        a = actions.permute(1, 0, 2).reshape(B, -1)
        return torch.cat([s, a], 1)

    def learn(self, states, actions, rewards, next_states, dones, u_next=None, u_cur=None, critic_in=None):
        """One MADDPG update from a sampled batch.  states/next_states [K, B, H, W] f32, actions
        [K, B, 9] (stored GumbelSoftmax probabilities), rewards [B, K], dones [B, K] (termination).
        u_next / u_cur: optional uniforms [K, B, 9] for the two Gumbel samples (tests).
        critic_in: optional (x, x_next) critic input rows from ReplayRing.sample(critic_in=True)
        (GPU): the same values this method would assemble, without the permute / cat copies.
        With several ranks each backward is followed by the gradient all-reduce.
        Returns (actor_loss [K], critic_loss [K]) device tensors (no host sync)."""
        ctx = self._learn_critic(states, actions, rewards, next_states, dones, u_next, critic_in)
        self._allreduce_grads("critic")
        self._learn_actor(ctx, u_cur)
        self._allreduce_grads("actor")
        self._desc_stale = True  # weights changed outside the descriptor learner
        return self._learn_finish(ctx)

    # ---- the descriptor learner (csrc/maddpg_ops.hip gw_maddpg_desc_update) -------------------
    def desc_capable(self, replay, generator=None) -> bool:
        """Whether an update on ``replay`` can run as the descriptor learner: one rank, the fused
        flat networks with in-kernel draws, a ReplayRing currently serving descriptor rows, a batch
        of 16..256 rows in 16-row tiles (GW_DESC_LEARN=0: never)."""
        import os
        return (generator is None and self.device.type == "cuda" and self.world <= 1 and self._draws_in_kernel()
                and getattr(replay, "use_desc", False) and 16 <= self.batch_size <= 256
                and self.batch_size % 16 == 0 and self.K <= _lib.GW_MAX_AGENTS and replay.K == self.K
                and tuple(replay.obs.shape[-2:]) == (self.H, self.W) and os.environ.get("GW_DESC_LEARN", "1") != "0")

    def _desc_setup(self, replay) -> dict:
        """The descriptor learner's buffers and ABI structs for ``replay`` (built once per ring)."""
        d = self._desc.get(id(replay))
        if d is not None and d["replay"] is replay:
            return d
        L = _lib.load()
        B = self.batch_size
        n = int(L.gw_maddpg_desc_workspace_floats(self.K, B, self.H, self.W))
        if n < 0:
            raise ValueError("gw_maddpg_desc_workspace_floats: bad shape")
        ring = _lib.GwDescRing(replay.desc.data_ptr(), replay.probs.data_ptr(), replay.reward.data_ptr(),
                               replay.term.data_ptr(), replay.done.data_ptr(), replay.t_dev.data_ptr(), replay.S)

        def adam(opt: FlatAdam):
            return _lib.GwAdamBuf(opt.flat.data_ptr(), opt.flat.grad.data_ptr(), opt.m.data_ptr(), opt.v.data_ptr(),
                                  opt.count.data_ptr(), opt.flat.numel(), opt.lr, opt.betas[0], opt.betas[1], opt.eps)
        d = dict(replay=replay, ws=torch.zeros(n, dtype=torch.float32, device=self.device), ring=ring,
                 specs=(_mlp_spec(self.actors.net), _mlp_spec(self.actor_targets.net), _mlp_spec(self.critics),
                        _mlp_spec(self.critic_targets)),
                 adam=(adam(self.opt_actor), adam(self.opt_critic)),
                 loss=(torch.zeros(self.K, dtype=torch.float32, device=self.device),
                       torch.zeros(self.K, dtype=torch.float32, device=self.device)))
        self._desc = {id(replay): d}
        self._desc_stale = True
        return d

    def desc_prime(self, replay):
        """Derive the descriptor learner's c1 partial sums from the current weights (enqueued)."""
        import ctypes as C
        d = self._desc_setup(replay)
        a, at, c, ct = d["specs"]
        _lib.check(_lib.load().gw_maddpg_desc_prime(C.byref(replay._src), C.byref(a), C.byref(at), C.byref(c),
                                                     C.byref(ct), self.batch_size, d["ws"].data_ptr(),
                                                     torch.cuda.current_stream(self.device).cuda_stream),
                   "gw_maddpg_desc_prime")
        self._desc_stale = False

    def _actor_images(self, env):
        """The fused actor's workspace parts for ``env`` (gw_actor_images_view) when its fused MLP
        path already acts on ``env`` (full-grid input), else None."""
        import ctypes as C
        st = getattr(self.actors, "_fast", None)
        if (env is None or self.actors.arch != "mlp" or st is None or st.get("env") is not env or st.get("patch", 0)
                or st.get("spec") is None):
            return None
        ws = st["ws"]
        key = (ws.data_ptr(), env.H * env.W, self.K)
        cached = getattr(self, "_img_view", None)
        if cached is None or cached[0] != key:
            im = _lib.GwActorImages()
            _lib.check(_lib.load().gw_actor_images_view(ws.data_ptr(), env.H * env.W, self.K, C.byref(im)),
                       "gw_actor_images_view")
            self._img_view = cached = (key, im, ws)
        return cached[1]

    def learn_desc(self, replay, actor_env=None):
        """One whole MADDPG update sampling the descriptor ring ``replay`` in four launches
        (gw_maddpg_desc_update): the sample, both gradients with their Adam steps and both soft
        target updates.  actor_env: an env the fused MLP actor acts on; the update then also leaves
        that actor's workspace parts (gw_maddpg_desc_update_img: row slices, W2 / W3 images), so
        the next act_env needs no gw_actor_prepare.  Returns (actor_loss [K], critic_loss [K])."""
        import ctypes as C
        d = self._desc_setup(replay)
        if self._desc_stale:
            self.desc_prime(replay)
        a, at, c, ct = d["specs"]
        oa, oc = d["adam"]
        la, lc = d["loss"]
        im = self._actor_images(actor_env)
        _lib.check(_lib.load().gw_maddpg_desc_update_img(
            C.byref(replay._src), C.byref(d["ring"]), C.byref(a), C.byref(at), C.byref(c), C.byref(ct), C.byref(oa),
            C.byref(oc), self.actor_targets.net.flat_params().data_ptr(), self.critic_targets.flat_params().data_ptr(),
            float(self.gamma), float(self.tau), self.batch_size, self._draw_key, d["ws"].data_ptr(), la.data_ptr(),
            lc.data_ptr(), C.byref(im) if im is not None else None, getattr(replay, "env_handle", None),
            torch.cuda.current_stream(self.device).cuda_stream), "gw_maddpg_desc_update")
        for net in (self.actors.net, self.critics, self.actor_targets.net, self.critic_targets):
            net.epoch += 1
        if im is not None and not torch.cuda.is_current_stream_capturing():
            # (inside a graph capture nothing ran yet: replay_learn marks each replay's workspace)
            self.actors.mark_prepared(actor_env)
        return la, lc

    def desc_records(self, replay) -> dict:
        """The last descriptor update's rows as the workspace holds them (tests): ``idx`` [B, 2]
        (transition slot, env), the Gumbel uniforms ``u_next`` / ``u_cur`` [K, B, 9], the target
        actions ``a_next`` [B, 9K] (synchronises)."""
        d = self._desc_setup(replay)
        ws, K, B = d["ws"], self.K, self.batch_size
        r4 = lambda n: (n + 3) // 4 * 4  # noqa: E731  (csrc dws_layout's 16-byte rounding)
        npm = _lib.GW_MAX_AGENTS + 1     # patch slots per (row, agent obs)
        o = 0
        idx = ws[o:o + 2 * B].view(torch.int32).reshape(B, 2)
        o += r4(2 * B) + 2 * r4(2 * K * B * npm) + r4(2 * K * B)
        o += r4(B * 9 * K)  # act
        tact = ws[o:o + B * 9 * K].reshape(B, 9 * K)
        o += r4(B * 9 * K)
        u = ws[o:o + 2 * K * B * 9].reshape(2, K, B, 9)
        return {"idx": idx.clone(), "u_next": u[0].clone(), "u_cur": u[1].clone(), "a_next": tact.clone()}

    def _fused_batch(self, x, x_next, rewards, dones, u):
        """u None: the kernels draw the Gumbel uniforms (Philox keyed by _draw_key and the critic
        optimizer's step count)."""
        return _lib.GwMaddpgBatch(self.K, x.shape[0], self.H * self.W, x.data_ptr(), x_next.data_ptr(), rewards.data_ptr(),
                                  dones.data_ptr(), u.data_ptr() if u is not None else None, self._draw_key,
                                  self.opt_critic.count.data_ptr() if u is None else None)

    def _draws_in_kernel(self) -> bool:
        """Whether the fused update draws its randomness itself (GPU, flat Adam step counts)."""
        return self.fused and isinstance(self.opt_critic, FlatAdam)

    def _fused_ws(self, B: int) -> torch.Tensor:
        ws = self._fws.get(B)
        if ws is None:
            n = int(_lib.load().gw_maddpg_workspace_floats(self.K, B, self.H * self.W))
            ws = self._fws[B] = torch.empty(n, dtype=torch.float32, device=self.device)
        return ws

    def _fused_critic(self, states, actions, rewards, next_states, dones, u_next, critic_in) -> dict:
        """Phase 1 as gw_maddpg_critic_grads (include/learner_ops.h): 3 launches."""
        import ctypes as C
        K, B = states.shape[0], states.shape[1]
        dev = self.device
        if critic_in is not None:
            x, x_next = critic_in
        else:
            x = self._critic_in(states, actions)
            x_next = self._critic_in(next_states, torch.zeros_like(actions))
        x, x_next = x.contiguous(), x_next.contiguous()
        if not (x.dtype == x_next.dtype == torch.float32 and tuple(x.shape) == tuple(x_next.shape)
                == (B, K * self.H * self.W + K * N_ACTIONS)):
            raise ValueError("critic input rows must be float32 [B, K*H*W + K*9]")
        if u_next is not None:
            u = u_next.to(torch.float32).contiguous()
        else:
            u = None if self._draws_in_kernel() else torch.rand((K, B, N_ACTIONS), device=dev)
        r = rewards.to(device=dev, dtype=torch.float64).contiguous()
        d = dones.to(device=dev, dtype=torch.uint8).contiguous()
        loss = torch.empty((K,), dtype=torch.float32, device=dev)
        ws = self._fused_ws(B)
        batch = self._fused_batch(x, x_next, r, d, u)
        at, ct, c = _mlp_spec(self.actor_targets.net), _mlp_spec(self.critic_targets), _mlp_spec(self.critics)
        cg = _mlp_spec(self.critics, grad=True)
        _lib.check(_lib.load().gw_maddpg_critic_grads(C.byref(at), C.byref(ct), C.byref(c), C.byref(cg), C.byref(batch),
                                                      float(self.gamma), ws.data_ptr(), loss.data_ptr(),
                                                      self._count_ptr(self.opt_critic),
                                                      torch.cuda.current_stream(dev).cuda_stream),
                   "gw_maddpg_critic_grads")
        return dict(fused=True, x=x, x_next=x_next, r=r, d=d, u_next=u, states=states, critic_loss=loss, B=B)

    @staticmethod
    def _count_ptr(opt):
        """The FlatAdam step count the fused gradient launch advances (its Adam step then only
        reads it: no arrival counter); None for another optimizer."""
        return opt.count.data_ptr() if isinstance(opt, FlatAdam) else None

    def _fused_actor(self, ctx: dict, u_cur=None):
        """Phase 2 (after the critic's Adam step) as gw_maddpg_actor_grads: 3 launches."""
        import ctypes as C
        K, B, dev = self.K, ctx["B"], self.device
        if u_cur is not None:
            u = u_cur.to(torch.float32).contiguous()
        else:
            u = None if self._draws_in_kernel() else torch.rand((K, B, N_ACTIONS), device=dev)
        loss = torch.empty((K,), dtype=torch.float32, device=dev)
        batch = self._fused_batch(ctx["x"], ctx["x_next"], ctx["r"], ctx["d"], u)
        a, c, ag = _mlp_spec(self.actors.net), _mlp_spec(self.critics), _mlp_spec(self.actors.net, grad=True)
        _lib.check(_lib.load().gw_maddpg_actor_grads(C.byref(a), C.byref(c), C.byref(ag), C.byref(batch),
                                                     self._fused_ws(B).data_ptr(), loss.data_ptr(), None,
                                                     self._count_ptr(self.opt_actor),
                                                     torch.cuda.current_stream(dev).cuda_stream),
                   "gw_maddpg_actor_grads")
        ctx["u_cur"] = u
        ctx["actor_loss"] = loss

    def _learn_critic(self, states, actions, rewards, next_states, dones, u_next=None, critic_in=None) -> dict:
        """Phase 1: target actions, TD target, critic forward and backward (gradients in the
        critics' .grad, not yet applied)."""
        K, B = states.shape[0], states.shape[1]
        # the fused kernels take batches of 16-row tiles (gw_maddpg_* reject B % 16 != 0) and at
        # most GW_MAX_AGENTS agents; any other batch runs the torch composition
        if self.fused and B >= 16 and B % 16 == 0 and K <= _lib.GW_MAX_AGENTS:
            return self._fused_critic(states, actions, rewards, next_states, dones, u_next, critic_in)
        D = K * self.H * self.W
        with torch.no_grad():
            if critic_in is not None:
                x, x_next = critic_in
                _gumbel_into_slots(self.actor_targets(next_states), u_next, x_next, D)
            else:
                logits = self.actor_targets(next_states)
                a_next = _gumbel_hip(logits, u_next) if self.flat else gumbel_softmax(logits, u_next)  # [K, B, 9]
                x_next = self._critic_in(next_states, a_next)
            q_next = self.critic_targets(x_next.unsqueeze(0).expand(K, -1, -1))     # [K, B, 1]
            y = self._td_target(rewards, dones, q_next)
        if critic_in is None:
            x = self._critic_in(states, actions)
        q = self.critics(x.unsqueeze(0).expand(K, -1, -1))
        if self.flat:
            critic_loss = _MeanLoss.apply(q, y, 0)                                    # MSELoss per agent
        else:
            critic_loss = ((q - y) ** 2).mean(dim=(1, 2))
        self.opt_critic.zero_grad(set_to_none=False)
        critic_loss.sum().backward()
        return dict(states=states, actions=actions, x=x, critic_loss=critic_loss.detach())

    def _learn_actor(self, ctx: dict, u_cur=None):
        """Phase 2: the critic's Adam step, then the actor loss through the updated critics and
        its backward (gradients in the actors' .grad, not yet applied)."""
        if isinstance(self.opt_critic, FlatAdam):
            self.opt_critic.step(advanced=bool(ctx.get("fused")))
        else:
            self.opt_critic.step()
        if ctx.get("fused"):
            self._fused_actor(ctx, u_cur)
            return
        states, actions, x = ctx["states"], ctx["actions"], ctx["x"]
        K, B = states.shape[0], states.shape[1]
        probs = gumbel_softmax(self.actors(states), u_cur)                             # [K, B, 9]
        # a_mix[k] = the replayed actions with agent k's slot replaced by its fresh probs
        a_mix = actions.permute(1, 0, 2).unsqueeze(0).repeat(K, 1, 1, 1)              # [K, B, K, 9]
        a_mix.diagonal(dim1=0, dim2=2).copy_(probs.permute(1, 2, 0))
        # The actor loss needs gradients for the actors only: the critics' parameter
        # gradients this backward would form are dead (zeroed before the next critic step),
        # so the critics enter as constants, and critic layer 1 is split into its state
        # columns (no gradient path) and its action columns (the only path to the actors).
        qa = self._q_split(x, a_mix.reshape(K, B, -1))
        actor_loss = _MeanLoss.apply(qa, None, 1) if self.flat else -qa.mean(dim=(1, 2))
        self.opt_actor.zero_grad(set_to_none=False)
        actor_loss.sum().backward()
        ctx["actor_loss"] = actor_loss.detach()

    def _learn_finish(self, ctx: dict):
        """Phase 3: the actor's Adam step and the soft target update (flat buffers: one launch)."""
        if self.flat and isinstance(self.opt_actor, FlatAdam):
            t1 = self.actor_targets.net.flat_params()
            t2, p2 = self.critic_targets.flat_params(), self.critics.flat_params()
            with torch.no_grad():
                self.opt_actor.step_soft(t1, self.tau, t2, p2, advanced=bool(ctx.get("fused")))
            self.actor_targets.net.epoch += 1
            self.critic_targets.epoch += 1
        else:
            self.opt_actor.step()
            self.soft_update()
        return ctx["actor_loss"], ctx["critic_loss"]

    def _q_split(self, x: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
        """Q_k of the critics as constants on rows whose state columns are x[:, :D] and whose action
        columns are a [K, B, K*9] (per agent k): critic layer 1 as a state-column GEMM plus an
        action-column GEMM.  The same function as critics(cat(x[:, :D], a_k)); the split changes
        layer 1's summation order (two partial sums instead of one), so Q differs from the
        concatenated forward by f32 rounding only (tests/test_maddpg.py::test_split_q_matches_concat_q)."""
        K, B = a.shape[0], a.shape[1]
        D = K * self.H * self.W
        c = self.critics
        w1 = c.weights[0].detach()
        z1 = torch.baddbmm(c.biases[0].detach(), x[:, :D].detach().unsqueeze(0).expand(K, -1, -1), w1[:, :D])
        z1 = torch.baddbmm(z1, a, w1[:, D:])
        return c(z1, pre=True, frozen=True)

    def _td_target(self, rewards, dones, q_next):
        """y = r + (1 - d) * gamma * q_next  ([K, B, 1]; rewards f64 / dones [B, K])."""
        if self.flat and rewards.dtype == torch.float64 and dones.dtype == torch.uint8:
            q_next = q_next.contiguous()
            y = torch.empty_like(q_next)
            _lib.check(_lib.load().gw_td_target(rewards.contiguous().data_ptr(), dones.contiguous().data_ptr(),
                                                q_next.data_ptr(), self.gamma, y.data_ptr(), q_next.shape[0],
                                                q_next.shape[1], torch.cuda.current_stream(self.device).cuda_stream),
                       "gw_td_target")
            return y
        r = rewards.to(torch.float32).t().unsqueeze(-1)          # [K, B, 1]
        d = dones.to(torch.float32).t().unsqueeze(-1)
        return r + (1.0 - d) * self.gamma * q_next

    @torch.no_grad()
    def soft_update(self):
        """agilerl soft_update: target <- tau * online + (1 - tau) * target (flat: one gw_soft_update
        launch per network; otherwise two foreach kernels)."""
        if self.flat:
            s = torch.cuda.current_stream(self.device).cuda_stream
            t1, p1 = self.actor_targets.net.flat_params(), self.actors.net.flat_params()
            t2, p2 = self.critic_targets.flat_params(), self.critics.flat_params()
            _lib.check(_lib.load().gw_soft_update2(t1.data_ptr(), p1.data_ptr(), t1.numel(), t2.data_ptr(),
                                                   p2.data_ptr(), t2.numel(), self.tau, s), "gw_soft_update2")
            self.actor_targets.net.epoch += 1
            self.critic_targets.epoch += 1
            return
        src = list(self.actors.parameters()) + list(self.critics.parameters())
        dst = list(self.actor_targets.parameters()) + list(self.critic_targets.parameters())
        torch._foreach_mul_(dst, 1.0 - self.tau)
        torch._foreach_add_(dst, src, alpha=self.tau)

    # ---------------------------------------------------------------------------------------
    def learn_from(self, replay, generator: torch.Generator | None = None):
        """Sample ``batch_size`` transitions from a ReplayRing and learn (eager): the descriptor
        learner where it applies (desc_capable), else the sample launch + ``learn``."""
        if self.desc_capable(replay, generator):
            return self.learn_desc(replay)
        return self.learn(*self._sample(replay, generator))

    def _sample(self, replay, generator=None):
        """(states, actions, rewards, next_states, dones, u_next, u_cur, critic_in) as ``learn``
        takes them (no explicit uniforms; critic_in from the gather launch on the GPU)."""
        if self.device.type == "cuda" and generator is None and self._draws_in_kernel() \
                and self.batch_size % 16 == 0 and self.K <= _lib.GW_MAX_AGENTS:
            # the fused update: the sample's rows and both Gumbel samples' uniforms are drawn
            # inside the gather launch and the tails (Philox, no torch RNG launch)
            *batch, ci = replay.sample(self.batch_size, critic_in=True,
                                       philox=(self._draw_key, self.opt_critic.count))
            return (*batch, None, None, ci)
        if self.device.type == "cuda":  # the critic's input rows come from the gather launch
            # the two Gumbel samples' uniforms come from the sample's own torch.rand launch
            n = self.K * self.batch_size * N_ACTIONS
            *batch, ci, uu = replay.sample(self.batch_size, generator=generator, critic_in=True, extra_uniform=2 * n)
            shape = (self.K, self.batch_size, N_ACTIONS)
            return (*batch, uu[:n].view(shape), uu[n:].view(shape), ci)
        return (*replay.sample(self.batch_size, generator=generator), None, None, None)

    def capture(self, replay=None, warmup: int = 3, batch: tuple | None = None, actor_env=None,
                launches: bool = False):
        """Capture sample + learn into HIP graphs (requires capturable=True and a CUDA device).
        Later ``replay_learn()`` replays them.  ``batch`` (instead of a ReplayRing): fixed input
        tensors (states, actions, rewards, next_states, dones[, u_next, u_cur]) the graphs read
        at every replay.  One rank: ONE graph (one launch instead of ~150 kernel launches).
        Several ranks: three graph segments sharing one memory pool (sample + critic backward |
        critic step + actor backward | actor step + soft update) with the two gradient
        all-reduces issued eagerly between their replays (a collective is not captured: the gloo
        backend cannot be, and RCCL's own launches stay outside the graph).
        actor_env: the env the fused actors act on; the graph then ends with the actors' workspace
        derivation for it (one rank), so the next act_env after a replay needs no host round trip.
        launches (one rank, the fused update sampling ``replay`` with in-kernel draws; ignored
        otherwise): record the C-ABI launches of one more eager update (_lib.LaunchRecorder; it
        runs) and have replay_learn re-issue them on the current stream instead of a graph
        replay: no wait on a graph's completion before the next launch (profiles/r4_ab)."""
        if self.device.type != "cuda":
            raise RuntimeError("graph capture needs the GPU")
        # which rows the captured sample reads (the descriptor ring or the dense obs slots): the
        # caller's fence must match it, and a change of the ring's mode invalidates the capture
        self._capture_desc = bool(getattr(replay, "use_desc", False)) if batch is None else None
        desc = batch is None and self.desc_capable(replay)
        # which learner the capture holds: replay_learn primes / marks staleness only for the
        # descriptor learner's capture, not whenever _desc happens to be populated
        self._capture_is_desc = bool(desc)
        if desc:
            return self._capture_desc_learner(replay, warmup, actor_env, launches)
        if batch is not None:
            fixed = tuple(batch) + (None,) * (8 - len(batch))

            def draw():
                return fixed
        else:
            def draw():
                return self._sample(replay)
        # launches: only where every launch of the update goes through the C ABI (the fused update
        # sampling a ReplayRing with in-kernel draws: no torch kernel to miss); else the graph
        launches = launches and self.world <= 1 and batch is None and self._draws_in_kernel() and \
            self.batch_size % 16 == 0 and self.K <= _lib.GW_MAX_AGENTS
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            # allocator + optimizer state warm-up outside the graph (the recorded update below is
            # the last warm-up update when recording launches)
            for _ in range(max(0, warmup - 1) if launches else warmup):
                self.learn(*draw())
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.world <= 1:
            self._prep_env = self._prep_ws = None
            self._launches = None
            if launches:
                # recorded from one more eager update (it runs): its buffers come from the ordinary
                # allocator and are held here for as long as the recording is replayed
                rec = _lib.LaunchRecorder(torch.cuda.current_stream(self.device).cuda_stream)
                with rec:
                    b = draw()
                    st, ac, rw, ns, dn, un, uc, ci = b
                    ctx = self._learn_critic(st, ac, rw, ns, dn, un, ci)
                    self._learn_actor(ctx, uc)
                    self._graph_out = self._learn_finish(ctx)
                    if actor_env is not None:
                        self._prep_ws = self.actors.prepare_after_update(actor_env)
                        self._prep_env = actor_env if self._prep_ws is not None else None
                for m in (self.actors, self.actor_targets):
                    m.mark_updated()
                if self._prep_env is not None:
                    self.actors.mark_prepared(self._prep_env)
                self._launch_keep = (b, ctx)
                self._graph = self._launches = rec
                return rec
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._graph_out = self.learn(*draw())
                if actor_env is not None:
                    # the graph writes this workspace on every replay: hold it as long as the graph
                    self._prep_ws = self.actors.prepare_after_update(actor_env)
                    self._prep_env = actor_env if self._prep_ws is not None else None
            self._graph = g
            return g
        g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            st, ac, rw, ns, dn, un, uc, ci = draw()
            ctx = self._learn_critic(st, ac, rw, ns, dn, un, ci)
        with torch.cuda.graph(g2, pool=g1.pool()):
            self._learn_actor(ctx, uc)
        with torch.cuda.graph(g3, pool=g1.pool()):
            self._graph_out = self._learn_finish(ctx)
        self._graph_ctx = ctx  # keeps the segments' shared tensors alive
        self._graphs = (g1, g2, g3)
        self._graph = g3
        return g3

    def _capture_desc_learner(self, replay, warmup: int, actor_env, launches: bool):
        """capture() for the descriptor learner: its update is ONE C-ABI call (four launches),
        recorded (launches) or captured into a HIP graph, after the same warm-up updates."""
        for _ in range(max(0, warmup - 1) if launches else warmup):
            self.learn_desc(replay)
        if self._desc_stale:
            self.desc_prime(replay)  # outside the recording: replays then never prime
        self._prep_env = self._prep_ws = None
        self._launches = None
        fused_prep = self._actor_images(actor_env) is not None  # the update leaves the actor's workspace
        if launches:
            rec = _lib.LaunchRecorder(torch.cuda.current_stream(self.device).cuda_stream)
            with rec:
                self._graph_out = self.learn_desc(replay, actor_env=actor_env)
                if fused_prep:
                    self._prep_ws, self._prep_env = self.actors._fast["ws"], actor_env
                elif actor_env is not None:
                    self._prep_ws = self.actors.prepare_after_update(actor_env)
                    self._prep_env = actor_env if self._prep_ws is not None else None
            for m in (self.actors, self.actor_targets):
                m.mark_updated()
            if self._prep_env is not None:
                self.actors.mark_prepared(self._prep_env)
            self._launch_keep = None
            self._graph = self._launches = rec
            return rec
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                self._graph_out = self.learn_desc(replay, actor_env=actor_env)
                if fused_prep:
                    self._prep_ws, self._prep_env = self.actors._fast["ws"], actor_env
                elif actor_env is not None:
                    self._prep_ws = self.actors.prepare_after_update(actor_env)
                    self._prep_env = actor_env if self._prep_ws is not None else None
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._graph = g
        return g

    def invalidate_capture(self):
        """Drop the captured update (graph, segments or recorded launches): the next learn through
        a trainer captures again, e.g. after the replay ring switched between descriptor and dense
        rows (Rollout.reset / resume)."""
        self._graph = self._graphs = self._launches = None
        self._launch_keep = self._graph_ctx = None
        self._prep_env = self._prep_ws = None
        self._capture_desc = None
        self._capture_is_desc = False

    def capture_matches(self, replay) -> bool:
        """Whether the captured update samples the rows ``replay`` currently offers."""
        return self._graph is not None and getattr(self, "_capture_desc", None) == bool(getattr(replay, "use_desc", False))

    def replay_learn(self):
        desc = getattr(self, "_capture_is_desc", False) and self._desc
        if desc and self._desc_stale:
            # weights changed since the capture (a load, a dense update): re-derive the partial sums
            self.desc_prime(next(iter(self._desc.values()))["replay"])
        if self._graphs is not None:
            g1, g2, g3 = self._graphs
            g1.replay()
            self._allreduce_grads("critic")
            g2.replay()
            self._allreduce_grads("actor")
            g3.replay()
        elif getattr(self, "_launches", None) is not None:
            self._launches.replay(torch.cuda.current_stream(self.device).cuda_stream)
        else:
            self._graph.replay()
        for m in (self.actors, self.actor_targets):  # the replayed optimizer / soft update wrote them
            m.mark_updated()
        if self._graphs is None and getattr(self, "_prep_env", None) is not None:
            self.actors.mark_prepared(self._prep_env)  # the graph ended with the workspace derivation
        if not desc:
            self._desc_stale = True
        return self._graph_out

    # ---------------------------------------------------------------------------------------
    def state_dict(self) -> dict:
        """Flat tensor dict in the checkpoint naming (per agent), for safetensors."""
        out = {}
        for name, m in (("actor", self.actors), ("actor_target", self.actor_targets), ("critic", self.critics),
                        ("critic_target", self.critic_targets)):
            for k, v in m.state_dict().items():
                out[f"{name}.{k}"] = v.detach().contiguous()
        return out

    def load_state_dict(self, sd: dict):
        for name, m in (("actor", self.actors), ("actor_target", self.actor_targets), ("critic", self.critics),
                        ("critic_target", self.critic_targets)):
            sub = {k[len(name) + 1:]: v for k, v in sd.items() if k.startswith(name + ".")}
            m.load_state_dict(sub)
        self._desc_stale = True

    def optim_state_dict(self) -> dict:
        """The two optimizers' state as flat tensors (agilerl's save_checkpoint keeps the optimizer
        state dicts beside the networks): FlatAdam's moments and step count, or torch Adam's
        per-parameter exp_avg / exp_avg_sq / step in parameter order."""
        out = {}
        for name, opt in (("opt_actor", self.opt_actor), ("opt_critic", self.opt_critic)):
            if isinstance(opt, FlatAdam):
                out[f"{name}.m"], out[f"{name}.v"], out[f"{name}.count"] = opt.m, opt.v, opt.count
                continue
            for i, p in enumerate(opt.param_groups[0]["params"]):
                st = opt.state.get(p)
                if not st:
                    continue
                for key in ("exp_avg", "exp_avg_sq", "step"):
                    out[f"{name}.{i}.{key}"] = torch.as_tensor(st[key])
        return {k: v.detach().contiguous() for k, v in out.items()}

    @torch.no_grad()
    def load_optim_state_dict(self, sd: dict):
        for name, opt in (("opt_actor", self.opt_actor), ("opt_critic", self.opt_critic)):
            if isinstance(opt, FlatAdam):
                if f"{name}.m" in sd:
                    opt.m.copy_(sd[f"{name}.m"])
                    opt.v.copy_(sd[f"{name}.v"])
                    c = sd[f"{name}.count"].reshape(-1)  # round-3 checkpoints: [1] (no arrival counter)
                    opt.count.zero_()
                    opt.count[: c.numel()].copy_(c)
                continue
            for i, p in enumerate(opt.param_groups[0]["params"]):
                if f"{name}.{i}.exp_avg" not in sd:
                    continue
                st = opt.state.get(p)
                if st and all(isinstance(st.get(key), torch.Tensor) for key in ("exp_avg", "exp_avg_sq", "step")):
                    # in place: a captured update graph (capturable Adam) keeps reading and writing
                    # these very tensors, so replacing them would silently detach it from the load
                    for key in ("exp_avg", "exp_avg_sq", "step"):
                        st[key].copy_(sd[f"{name}.{i}.{key}"])
                else:
                    opt.state[p] = {key: sd[f"{name}.{i}.{key}"].to(p.device if key != "step" else
                                                                         sd[f"{name}.{i}.step"].device).clone()
                                    for key in ("exp_avg", "exp_avg_sq", "step")}

    def save(self, path: str, optimizer: bool = True):
        """Networks (+ optimizer state) as safetensors."""
        from safetensors.torch import save_file
        sd = dict(self.state_dict())
        if optimizer:
            sd.update(self.optim_state_dict())
        save_file({k: v.cpu() for k, v in sd.items()}, path)

    def load(self, path: str):
        from safetensors.torch import load_file
        sd = load_file(path)
        self.load_state_dict({k: v.to(self.device) for k, v in sd.items() if not k.startswith("opt_")})
        self.load_optim_state_dict({k: v.to(self.device) for k, v in sd.items() if k.startswith("opt_")})
        self.actors.mark_updated()


def learns_per_step(num_envs: int, learn_step: int, idx_step: int) -> int:
    """agilerl/MADDPGAgent.train learn schedule (maddpg/agent.py:199-224): with learn_step >
    num_envs, one learn every learn_step // num_envs env steps; otherwise num_envs // learn_step
    learns per env step."""
    if learn_step > num_envs:
        return 1 if idx_step % (learn_step // num_envs) == 0 else 0
    return num_envs // learn_step
