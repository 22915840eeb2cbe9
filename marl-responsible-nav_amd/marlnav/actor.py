"""MADDPG actors (PyTorch-ROCm), batched over envs and stacked over the K RL agents.

The reference drives one actor per RL agent through agilerl 1.0.15's MADDPG
(maddpg/agent.py:41-65, get_action at :109-113).  agilerl is not installed here; the actor
architecture is the one the shipped checkpoints hold:

  MLP  (configs/mlp.yaml):  Linear(H*W -> 128) - LayerNorm - ReLU - Linear(128 -> 128) - LayerNorm
                            - ReLU - Linear(128 -> 9) - GumbelSoftmax
  CNN  (configs/cnn.yaml):  Conv2d(1 -> 32, k2, s2) - ReLU - Conv2d(32 -> 64, k2, s2) - ReLU - flatten
                            - Linear(-> 128) - ReLU - Linear(128 -> 128) - ReLU - Linear(128 -> 9)

The K agents' MLPs run as one batched GEMM chain (torch.bmm over stacked [K, in, out] weights),
so a step is three GEMM launches for all agents instead of 3K.  Exploration: agilerl's
GumbelSoftmax sample during training, then invalid actions (the env's action mask) are
removed and the argmax is taken.  That sampling path is "parity unpinned" (agilerl is absent
and the reference has no test of it); the deterministic logits are a plain restatement.
"""
from __future__ import annotations

import ctypes as C
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

N_ACTIONS = 9


def _init_linear(K, fan_in, fan_out, gen=None):
    bound = 1.0 / math.sqrt(fan_in)  # nn.Linear's default (kaiming_uniform a=sqrt(5)) bound
    w = (torch.rand((K, fan_in, fan_out), generator=gen, device="cpu") * 2 - 1) * bound
    b = (torch.rand((K, 1, fan_out), generator=gen, device="cpu") * 2 - 1) * bound
    return w, b


class _LnRelu(torch.autograd.Function):
    """relu(ln_b + layer_norm(z) * ln_w) over [K, R, h] as the one-launch HIP epilogue
    (gw_ln_relu_fwd / gw_ln_relu_bwd, include/learner_ops.h).  The backward adds the ln_w / ln_b
    gradients straight into the parameters' preallocated .grad views of the flat gradient buffer
    (what autograd's accumulation would do, minus its add launches) and returns None for them."""

    @staticmethod
    def forward(ctx, z, ln_w, ln_b, save=True):
        # save: whether a backward can follow (grad mode is off inside forward, so the caller,
        # ln_relu(), decides)
        from . import _lib
        K, R, h = z.shape
        z = z.contiguous()
        y = torch.empty_like(z)
        stats = torch.empty((2, K, R), device=z.device, dtype=torch.float32) if save else None
        s = torch.cuda.current_stream(z.device).cuda_stream
        _lib.check(_lib.load().gw_ln_relu_fwd(z.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(), y.data_ptr(),
                                              stats[0].data_ptr() if save else None,
                                              stats[1].data_ptr() if save else None, K, R, h, 1e-5, s),
                   "gw_ln_relu_fwd")
        if save:
            ctx.save_for_backward(z, y, ln_w, stats)
            ctx.params = (ln_w, ln_b)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        z, y, ln_w, stats = ctx.saved_tensors
        K, R, h = z.shape
        dy = dy.contiguous()
        dz = torch.empty_like(z)
        out = []
        for i, p in enumerate(ctx.params):
            if not ctx.needs_input_grad[1 + i]:
                out.append((None, None))
            elif p.grad is not None and p.grad.is_contiguous():
                out.append((p.grad, None))  # accumulate in place, return None
            else:
                g = torch.zeros_like(p)
                out.append((g, g))
        s = torch.cuda.current_stream(z.device).cuda_stream
        _lib.check(_lib.load().gw_ln_relu_bwd(dy.data_ptr(), z.data_ptr(), y.data_ptr(), ln_w.data_ptr(),
                                              stats[0].data_ptr(), stats[1].data_ptr(), dz.data_ptr(),
                                              out[0][0].data_ptr() if out[0][0] is not None else None,
                                              out[1][0].data_ptr() if out[1][0] is not None else None,
                                              K, R, h, s), "gw_ln_relu_bwd")
        return (dz if ctx.needs_input_grad[0] else None), out[0][1], out[1][1], None


def ln_relu(z, ln_w, ln_b):
    """relu(ln_b + layer_norm(z) * ln_w) through the HIP epilogue (_LnRelu)."""
    save = torch.is_grad_enabled() and (z.requires_grad or ln_w.requires_grad or ln_b.requires_grad)
    return _LnRelu.apply(z, ln_w, ln_b, save)


class _AffineRelu(torch.autograd.Function):
    """relu(ln_b + xhat * ln_w) after torch's own F.layer_norm (gw_affine_relu_fwd / _bwd): the
    addcmul + relu and their backward (relu mask, addcmul's three products, the two row
    reductions and autograd's accumulation adds) as one launch each; the normalised rows are
    torch's, so the forward equals the torch composition bit for bit.  Parameter gradients are
    added into the preallocated .grad views like _LnRelu."""

    @staticmethod
    def forward(ctx, xhat, ln_w, ln_b, save=True):
        from . import _lib
        K, R, h = xhat.shape
        xhat = xhat.contiguous()
        y = torch.empty_like(xhat)
        _lib.check(_lib.load().gw_affine_relu_fwd(xhat.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(), y.data_ptr(), K, R,
                                                  h, torch.cuda.current_stream(xhat.device).cuda_stream),
                   "gw_affine_relu_fwd")
        if save:
            ctx.save_for_backward(xhat, y, ln_w)
            ctx.params = (ln_w, ln_b)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        xhat, y, ln_w = ctx.saved_tensors
        K, R, h = xhat.shape
        dy = dy.contiguous()
        dx = torch.empty_like(xhat) if ctx.needs_input_grad[0] else None
        out = []
        for i, p in enumerate(ctx.params):
            if not ctx.needs_input_grad[1 + i]:
                out.append((None, None))
            elif p.grad is not None and p.grad.is_contiguous():
                out.append((p.grad, None))
            else:
                g = torch.zeros_like(p)
                out.append((g, g))
        _lib.check(_lib.load().gw_affine_relu_bwd(
            dy.data_ptr(), xhat.data_ptr(), y.data_ptr(), ln_w.data_ptr(), dx.data_ptr() if dx is not None else None,
            out[0][0].data_ptr() if out[0][0] is not None else None,
            out[1][0].data_ptr() if out[1][0] is not None else None, K, R, h,
            torch.cuda.current_stream(xhat.device).cuda_stream), "gw_affine_relu_bwd")
        return dx, out[0][1], out[1][1], None


def affine_relu(xhat, ln_w, ln_b):
    save = torch.is_grad_enabled() and (xhat.requires_grad or ln_w.requires_grad or ln_b.requires_grad)
    return _AffineRelu.apply(xhat, ln_w, ln_b, save)


class _StackedLinear(torch.autograd.Function):
    """baddbmm(b, x, w) whose backward writes the parameter gradients straight into their
    preallocated .grad views: W.grad += x^T dy as ONE GEMM with beta = 1, b.grad += 1^T dy as
    another (autograd's version is GEMM + add and reduction + add)."""

    _ones = {}
    _ONES_MAX = 16

    @staticmethod
    def _ones_for(dy):
        """The cached [K, 1, R] ones of dy's shape.  Never created during a graph capture: there
        the fill kernel would only be recorded, and an eager backward before the first replay
        would read uninitialised memory; None then.  At most _ONES_MAX shapes are kept."""
        key = (dy.shape[0], dy.shape[1], dy.device, dy.dtype)
        ones = _StackedLinear._ones.get(key)
        if ones is None:
            if dy.is_cuda and torch.cuda.is_current_stream_capturing():
                return None
            if len(_StackedLinear._ones) >= _StackedLinear._ONES_MAX:
                _StackedLinear._ones.clear()
            ones = _StackedLinear._ones[key] = torch.ones((key[0], 1, key[1]), device=dy.device, dtype=dy.dtype)
        return ones

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.params = (w, b)
        return torch.baddbmm(b, x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        wp, bp = ctx.params
        dx = torch.bmm(dy, w.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        gw = gb = None
        if ctx.needs_input_grad[1]:
            if wp.grad is not None:
                wp.grad.baddbmm_(x.transpose(1, 2), dy)
            else:
                gw = torch.bmm(x.transpose(1, 2), dy)
        if ctx.needs_input_grad[2]:
            ones = _StackedLinear._ones_for(dy)
            if ones is None:  # inside a graph capture with no cached ones: a row sum instead
                if bp.grad is not None:
                    bp.grad.add_(dy.sum(1, keepdim=True))
                else:
                    gb = dy.sum(1, keepdim=True)
            elif bp.grad is not None:
                bp.grad.baddbmm_(ones, dy)
            else:
                gb = torch.bmm(ones, dy)
        return dx, gw, gb


def _linear_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and _AFFINE and torch.is_grad_enabled()


def _affine_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and _AFFINE


_AFFINE = __import__("os").environ.get("GW_AFFINE_FUSED", "1") != "0"


def _fused_ln_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and 0 < x.shape[-1] <= 512 and _FUSED_LN


# Opt-in (GW_LN_FUSED=1): the batch-128 update 0.817 -> 0.764 ms, but its row statistics round
# differently from torch's LayerNorm, so a ReLU mask at the rounding edge can flip and Adam's
# normalised step turns that into a visible parameter difference against the per-agent torch
# loop (tests/test_maddpg.py); the default keeps torch's LayerNorm on the learner path.
_FUSED_LN = __import__("os").environ.get("GW_LN_FUSED", "0") == "1"


class StackedMLPActors(nn.Module):
    """K independent MLPs evaluated together: x [K, E, D] -> [K, E, out] (out = 9 logits for an
    actor, 1 for a critic).

    The per-layer parameters ``weights[i]`` [K, in, out], ``biases[i]`` [K, 1, out], ``ln_w[i]`` /
    ``ln_b[i]`` [K, 1, h] are leaf Parameters that are views of ONE flat buffer, and
    ``flat_params()`` returns that buffer as a Parameter whose ``.grad`` is a flat gradient buffer
    the per-layer gradients accumulate into (in place).  An optimizer over the flat Parameter
    then takes one fused step per network, and the soft target update is one kernel: what
    bounds a batch-128 MADDPG update is launch count, not FLOPs."""

    def __init__(self, K: int, in_dim: int, hidden=(128, 128), n_actions: int = N_ACTIONS, layer_norm: bool = True,
                 device=None, dtype=torch.float32, seed: int = 0):
        super().__init__()
        gen = torch.Generator().manual_seed(seed)
        dims = [in_dim, *hidden, n_actions]
        parts, shapes = [], []
        for a, b in zip(dims[:-1], dims[1:]):
            w, bb = _init_linear(K, a, b, gen)
            parts += [w, bb]
            shapes += [("w", w.shape), ("b", bb.shape)]
        for h in hidden:
            parts += [torch.ones((K, 1, h)), torch.zeros((K, 1, h))]
            shapes += [("lw", (K, 1, h)), ("lb", (K, 1, h))]
        flat = torch.cat([t.reshape(-1) for t in parts]).to(device=device, dtype=dtype)
        # not registered: parameters() yields the per-layer views only (no double counting)
        object.__setattr__(self, "_flat", nn.Parameter(flat))
        self._flat.grad = torch.zeros_like(flat)
        lists = {"w": [], "b": [], "lw": [], "lb": []}
        off = 0
        for kind, shape in shapes:
            n = math.prod(shape)
            p = nn.Parameter(flat[off:off + n].view(shape))
            p.grad = self._flat.grad[off:off + n].view(shape)
            lists[kind].append(p)
            off += n
        self.weights = nn.ParameterList(lists["w"])
        self.biases = nn.ParameterList(lists["b"])
        self.ln_w = nn.ParameterList(lists["lw"])
        self.ln_b = nn.ParameterList(lists["lb"])
        self.layer_norm = layer_norm
        self.K, self.in_dim, self.n_layers = K, in_dim, len(dims) - 1
        self.epoch = 0  # bumped by writers that bypass torch's version counter (flat HIP Adam, soft update)

    def flat_params(self) -> nn.Parameter:
        """The single flat Parameter (shares storage with every layer; .grad = flat gradients)."""
        return self._flat

    def forward(self, x: torch.Tensor, pre: bool = False, frozen: bool = False) -> torch.Tensor:
        """pre: x is already layer 0's pre-activation (its GEMM + bias done by the caller).
        frozen: the parameters enter as constants (no parameter gradients are formed; gradients
        still flow to x)."""
        n = self.n_layers
        P = (lambda t: t.detach()) if frozen else (lambda t: t)
        for i in range(n):
            if i > 0 or not pre:
                if not frozen and _linear_ok(x) and self.weights[i].requires_grad:
                    x = _StackedLinear.apply(x, self.weights[i], self.biases[i])
                else:
                    x = torch.baddbmm(P(self.biases[i]), x, P(self.weights[i]))
            if i < n - 1:
                if self.layer_norm and _fused_ln_ok(x):  # one HIP launch (and one for its backward)
                    x = ln_relu(x, P(self.ln_w[i]), P(self.ln_b[i]))
                    continue
                if self.layer_norm and _affine_ok(x):  # torch's layer_norm, then one HIP launch
                    x = affine_relu(F.layer_norm(x, (x.shape[-1],)), P(self.ln_w[i]), P(self.ln_b[i]))
                    continue
                if self.layer_norm:  # nn.LayerNorm(h), eps 1e-5, per-agent affine
                    x = torch.addcmul(P(self.ln_b[i]), F.layer_norm(x, (x.shape[-1],)), P(self.ln_w[i]))
                x = F.relu(x)
        return x

    def load_agent(self, k: int, state: dict):
        """Per-agent weights in the checkpoint's naming (feature_net.linear_layer_i.weight [out, in], ...)."""
        names = [f"linear_layer_{i}" for i in range(self.n_layers - 1)] + ["linear_layer_output"]
        with torch.no_grad():
            for i, nm in enumerate(names):
                self.weights[i][k].copy_(torch.as_tensor(state[f"{nm}.weight"]).t())
                self.biases[i][k, 0].copy_(torch.as_tensor(state[f"{nm}.bias"]))
            for i in range(self.n_layers - 1):
                if f"layer_norm_{i}.weight" in state:
                    self.ln_w[i][k, 0].copy_(torch.as_tensor(state[f"layer_norm_{i}.weight"]))
                    self.ln_b[i][k, 0].copy_(torch.as_tensor(state[f"layer_norm_{i}.bias"]))


class CNNActor(nn.Module):
    """configs/cnn.yaml head for one agent: x [E, 1, H, W] -> logits [E, 9]."""

    def __init__(self, H: int, W: int, channels=(32, 64), kernels=(2, 2), strides=(2, 2), hidden=(128, 128),
                 n_actions: int = N_ACTIONS):
        super().__init__()
        layers, c, h, w = [], 1, H, W
        for ch, k, s in zip(channels, kernels, strides):
            layers += [nn.Conv2d(c, ch, k, s), nn.ReLU()]
            c, h, w = ch, (h - k) // s + 1, (w - k) // s + 1
        self.conv = nn.Sequential(*layers)
        dims = [c * h * w, *hidden]
        mlp = []
        for a, b in zip(dims[:-1], dims[1:]):
            mlp += [nn.Linear(a, b), nn.ReLU()]
        mlp.append(nn.Linear(dims[-1], n_actions))
        self.mlp = nn.Sequential(*mlp)

        # configs/cnn.yaml's convs have kernel == stride (non-overlapping 2x2 patches, no padding):
        # both convs are then per-patch GEMMs on hipBLASLt instead of MIOpen convolutions
        self.patchify = (len(channels) == 2 and all(k == s for k, s in zip(kernels, strides))
                         and H % (kernels[0] * kernels[1]) == 0 and W % (kernels[0] * kernels[1]) == 0)

    def fusable(self) -> bool:
        """configs/cnn.yaml exactly: conv 1 -> 32 -> 64, kernel 2 stride 2, hidden 128-128, 9 actions."""
        c1, c2 = self.conv[0], self.conv[2]
        return (len(self.conv) == 4 and c1.in_channels == 1 and c1.out_channels == 32 and c2.out_channels == 64
                and c1.kernel_size == (2, 2) and c1.stride == (2, 2) and c2.kernel_size == (2, 2)
                and c2.stride == (2, 2) and c1.padding == (0, 0) and c2.padding == (0, 0) and len(self.mlp) == 5
                and self.mlp[0].out_features == 128 and self.mlp[2].out_features == 128
                and self.mlp[4].out_features == N_ACTIONS)

    def forward(self, x):
        if self.patchify:
            return self._forward_patch_gemm(x)
        return self.mlp(self.conv(x).flatten(1))

    def _forward_patch_gemm(self, x):
        """Same function as ``conv -> flatten -> mlp`` (f32), with the two kernel == stride convs
        as GEMMs: obs pixels are grouped by conv-2 patch once, so conv 1's output rows are already
        conv 2's patch vectors (ky, kx, c order; the weights are permuted to match), and the
        flattened NHWC conv-2 output meets a column-permuted first Linear."""
        c1, c2 = self.conv[0], self.conv[2]
        k1, k2 = c1.kernel_size[0], c2.kernel_size[0]
        E, _, H, W = x.shape
        H2, W2 = H // (k1 * k2), W // (k1 * k2)
        # y = (k1 k2) y2 + k1 ky + py, x = (k1 k2) x2 + k1 kx + px
        p = x.reshape(E, H2, k2, k1, W2, k2, k1).permute(0, 1, 4, 2, 5, 3, 6).reshape(-1, k1 * k1)
        h = torch.relu(torch.addmm(c1.bias, p, c1.weight.reshape(c1.out_channels, -1).t()))
        h = h.reshape(E * H2 * W2, k2 * k2 * c1.out_channels)                 # (ky, kx, c) per patch
        w2 = c2.weight.permute(0, 2, 3, 1).reshape(c2.out_channels, -1)
        h = torch.relu(torch.addmm(c2.bias, h, w2.t())).reshape(E, -1)       # NHWC flatten
        lin = self.mlp[0]
        wl = lin.weight.reshape(lin.out_features, c2.out_channels, H2, W2).permute(0, 2, 3, 1).reshape(
            lin.out_features, -1)
        h = torch.relu(torch.addmm(lin.bias, h, wl.t()))
        return self.mlp[2:](h)


def _ctr_ptr(counter_dev):
    """Device address of the fused actors' noise-counter offset (a device int64 scalar) or None."""
    if counter_dev is None:
        return None
    if not (counter_dev.is_cuda and counter_dev.dtype == torch.int64 and counter_dev.numel() == 1):
        raise ValueError("counter_dev must be a device int64 scalar")
    return counter_dev.data_ptr()


class MultiAgentActors(nn.Module):
    """The K RL agents' actors: obs [K, E, H, W] -> logits [K, E, 9]."""

    def __init__(self, K: int, H: int, W: int, arch: str = "mlp", hidden=(128, 128), device=None,
                 dtype=torch.float32, seed: int = 0):
        super().__init__()
        self.K, self.H, self.W, self.arch, self.dtype = K, H, W, arch, dtype
        self._fast = None  # act_env's cached per-env state
        if arch == "mlp":
            self.net = StackedMLPActors(K, H * W, hidden, device=device, dtype=dtype, seed=seed)
        elif arch == "cnn":
            torch.manual_seed(seed)
            self.nets = nn.ModuleList([CNNActor(H, W, hidden=hidden) for _ in range(K)]).to(device=device, dtype=dtype)
        else:
            raise ValueError(arch)

    def forward(self, obs: torch.Tensor) -> torch.Tensor:
        K, E = obs.shape[0], obs.shape[1]
        x = obs.to(self.dtype)
        if self.arch == "mlp":
            return self.net(x.reshape(K, E, -1)).float()
        return torch.stack([self.nets[k](x[k].unsqueeze(1)) for k in range(K)]).float()

    @torch.no_grad()
    def act(self, obs: torch.Tensor, mask: torch.Tensor | None = None, training: bool = True,
            tau: float = 1.0, eps: float = 1e-20, generator: torch.Generator | None = None):
        """-> (actions [E, K] int32, probs [K, E, 9] float32 = the continuous actions stored in
        replay, as agilerl's MADDPG.get_action returns them)."""
        logits = self.forward(obs)
        if training:  # agilerl GumbelSoftmax: softmax((logits + Gumbel noise) / tau)
            u = torch.rand(logits.shape, device=logits.device, generator=generator)
            logits = logits - torch.log(-torch.log(u + eps) + eps)
        probs = torch.softmax(logits / tau, dim=-1)
        if mask is not None:  # env action mask [E, K] (9 bits) -> [K, E, 9]
            bits = (mask.t().to(torch.int32).unsqueeze(-1) >> torch.arange(N_ACTIONS, device=mask.device)) & 1
            probs_m = torch.where(bits.bool(), probs, torch.zeros((), device=probs.device))
        else:
            probs_m = probs
        actions = probs_m.argmax(-1).t().to(torch.int32).contiguous()
        return actions, probs

    # ---------------------------------------------------------------------------------------
    def fusable(self, env, patch: int = 0) -> bool:
        """The fused HIP get_action covers (gw_actor_act, include/actor_ops.h) the stacked f32 MLP
        with two 128-wide hidden layers and (gw_cnn_act) the configs/cnn.yaml CNN head, over a
        VecGridEnv's own observations; patch = P > 0: the MLP (gw_patch_actor_act) or the CNN head
        (gw_patch_cnn_act) over each agent's P x P window."""
        if self.dtype != torch.float32 or self.K != env.K:
            return False
        if patch and self.arch == "cnn":  # gw_patch_cnn_act
            return ((self.H, self.W) == (patch, patch) and patch in (4, 8, 12, 16) and env.H * env.W <= 4096
                    and all(n.fusable() for n in self.nets))
        if patch:
            net = getattr(self, "net", None)
            return (self.arch == "mlp" and (self.H, self.W) == (patch, patch) and env.H * env.W <= 4096
                    and net.n_layers == 3 and net.weights[0].shape[-1] == 128
                    and net.weights[1].shape == (self.K, 128, 128) and net.weights[2].shape[-1] == N_ACTIONS)
        if self.arch == "cnn":
            return ((self.H, self.W) == (env.H, env.W) and env.H % 4 == 0 and env.W % 4 == 0
                    and env.H * env.W <= 4096 and all(n.fusable() for n in self.nets))
        if self.arch != "mlp":
            return False
        net = self.net
        return (net.n_layers == 3 and net.weights[0].shape[-1] == 128 and net.weights[1].shape == (self.K, 128, 128)
                and net.weights[2].shape[-1] == N_ACTIONS and net.in_dim == env.H * env.W)

    def _ws_key(self):
        # the workspace (c1 = b1 + map . W1, W2/W3 operand images) is derived once per parameter
        # version: torch in-place ops bump the flat buffer's version counter, the HIP optimizer
        # (marlnav/maddpg.py) and graph replays bump net.epoch (mark_updated); every layer is a
        # view of the flat buffer, so its address pins the layer pointers
        flat = self.net.flat_params()
        return (flat._version, self.net.epoch, self.net.layer_norm, flat.data_ptr())

    def _prepare(self, env, st):
        """Enqueue the fused path's workspace derivation (gw_actor_prepare /
        gw_patch_actor_prepare) on the current stream."""
        from . import _lib
        net, K, dev, patch = self.net, self.K, env.device, st.get("patch", 0)
        ln = net.layer_norm
        ptrs = (net.weights[0], net.biases[0], net.ln_w[0], net.ln_b[0], net.weights[1], net.biases[1],
                net.ln_w[1], net.ln_b[1], net.weights[2], net.biases[2])
        st["spec"] = _lib.GwMlpActors(K, net.in_dim, 128, N_ACTIONS, int(ln),
                                      *[t.data_ptr() if (ln or i % 4 < 2 or i >= 8) else None
                                        for i, t in enumerate(ptrs)])
        with torch.cuda.device(dev):
            if patch:
                _lib.check(st["lib"].gw_patch_actor_prepare(env.handle, patch, C.byref(st["spec"]),
                                                            st["ws"].data_ptr(),
                                                            torch.cuda.current_stream(dev).cuda_stream),
                           "gw_patch_actor_prepare")
            else:
                _lib.check(st["lib"].gw_actor_prepare(env.handle, C.byref(st["spec"]), st["ws"].data_ptr(),
                                                      torch.cuda.current_stream(dev).cuda_stream),
                           "gw_actor_prepare")

    def prepare_after_update(self, env):
        """Enqueue the workspace derivation for ``env`` now, e.g. at the end of a captured update
        graph (after the optimizer step), so the next act_env starts on a fresh workspace without
        a host round trip; call ``mark_prepared(env)`` after each replay of that graph.  Only for
        an env the fused MLP path already acts on (act_env called once).  Returns the workspace
        tensor the enqueued launches write (a captured graph must hold it), or None."""
        st = self._fast
        if self.arch != "mlp" or st is None or st["env"] is not env or st.get("spec") is None:
            return None
        self._prepare(env, st)
        return st["ws"]

    def mark_prepared(self, env):
        """The workspace for ``env`` matches the current parameters (a replayed graph derived it)."""
        st = self._fast
        if st is not None and st["env"] is env:
            st["key"] = self._ws_key()

    def mark_updated(self):
        """Declare the parameters changed outside torch's in-place ops (HIP optimizer, graph
        replay): the fused path re-derives its workspace before the next act_env."""
        if self.arch == "mlp":
            self.net.epoch += 1
        else:
            self._epoch = getattr(self, "_epoch", 0) + 1

    def _mlp_workspace(self, env, patch: int):
        """The fused MLP path's per-(actors, env) state, its workspace derived for the current
        parameters (enqueued on the current stream when they changed)."""
        from . import _lib
        st = self._fast
        if st is None or st["env"] is not env or st.get("patch", 0) != patch:  # per-(actors, env) constants
            if not self.fusable(env, patch):
                raise _lib.GwError("act_env: actor not fusable (needs the f32 MLP 128-128-9 over the env's H*W obs, "
                                   "or over P x P windows with patch=P)")
            lib = _lib.load()
            ws_n = int(lib.gw_patch_actor_workspace_floats(patch, env.H, env.W, self.K) if patch
                       else lib.gw_actor_workspace_floats(self.net.in_dim, self.K))
            st = self._fast = dict(env=env, lib=lib, ws=torch.empty(ws_n, dtype=torch.float32, device=env.device),
                                   key=None, spec=None, actions=None, probs=None, patch=patch)
        key = self._ws_key()
        if key != st["key"]:
            self._prepare(env, st)
            st["key"] = key
        return st

    @torch.no_grad()
    def ensure_workspace(self, env, patch: int = 0):
        """Create and derive the fused path's workspace for ``env`` now, on the current stream.
        Rollout.capture calls it before capturing: a derivation (and the workspace's allocation)
        made inside a captured graph would run only in that graph's replays, so eager steps before
        the first replay would act on an underived workspace."""
        if self.arch == "cnn":
            self._cnn_workspace(env, int(patch))
        else:
            self._mlp_workspace(env, int(patch))

    @torch.no_grad()
    def act_env(self, env, mask: torch.Tensor | None = None, training: bool = True, tau: float = 1.0,
                seed: int = 0, counter: int = 0, uniform: torch.Tensor | None = None,
                actions_out: torch.Tensor | None = None, probs_out: torch.Tensor | None = None,
                logits_out: torch.Tensor | None = None, patch: int = 0, counter_dev: torch.Tensor | None = None,
                listed: bool = False):
        """``act`` on the observation ``env`` last wrote, as ONE fused HIP kernel (gw_actor_act):
        the first layer from the env's obs descriptors (map + patched cells, no obs read back),
        layers 2-3 on f32 MFMA, Gumbel noise from Philox(seed; env, counter, k) or ``uniform``
        [K, E, 9], softmax, mask, argmax.  -> (actions [E, K] int32, probs [K, E, 9] float32).
        counter_dev: a device int64 scalar added to ``counter`` when the kernel runs (the replay
        ring's step count: a captured graph's replays then draw fresh noise).
        patch = P > 0: actors built for P x P inputs act on each agent's egocentric window
        (gw_patch_actor_act; the windows VecGridEnv.obs_patch(P) would write).
        listed (the CNN head on windows): ``patch_cnn_write_list`` already listed the positions to
        recompute for the env's current descriptors on this stream (gw_patch_cnn_act_listed);
        ignored, and listed here again, when the workspace had to be re-derived first.
        Raises if the library or a GPU is missing (no fallback)."""
        from . import _lib
        if self.arch == "cnn":
            return self._act_env_cnn(env, mask, training, tau, seed, counter, uniform, actions_out, probs_out,
                                     logits_out, int(patch), counter_dev, listed)
        net, K, E, dev = self.net, self.K, env.E, env.device
        patch = int(patch)
        st = self._mlp_workspace(env, patch)
        if actions_out is None:
            actions_out = torch.empty((E, K), dtype=torch.int32, device=dev)
        if probs_out is None:
            probs_out = torch.empty((K, E, N_ACTIONS), dtype=torch.float32, device=dev)
        if not (actions_out.dtype == torch.int32 and actions_out.shape == (E, K) and actions_out.is_contiguous()):
            raise ValueError("act_env: actions_out must be a contiguous int32 [E, K] tensor")
        if not (probs_out.dtype == torch.float32 and probs_out.shape == (K, E, N_ACTIONS) and probs_out.is_contiguous()):
            raise ValueError("act_env: probs_out must be a contiguous float32 [K, E, 9] tensor")
        if uniform is not None and not (uniform.dtype == torch.float32 and uniform.shape == (K, E, N_ACTIONS)):
            raise ValueError("act_env: uniform must be float32 [K, E, 9]")
        if mask is not None and not (mask.shape == (E, K) and mask.element_size() == 2 and mask.is_contiguous()):
            raise ValueError("act_env: mask must be a contiguous 16-bit [E, K] tensor")
        args = (C.byref(st["spec"]), st["ws"].data_ptr(), int(bool(training)),
                float(tau), int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF,
                _ctr_ptr(counter_dev), uniform.contiguous().data_ptr() if uniform is not None else None,
                mask.data_ptr() if mask is not None else None, actions_out.data_ptr(), probs_out.data_ptr(),
                logits_out.data_ptr() if logits_out is not None else None, torch.cuda.current_stream(dev).cuda_stream)
        if patch:
            _lib.check(st["lib"].gw_patch_actor_act(env.handle, patch, *args), "gw_patch_actor_act")
        else:
            _lib.check(st["lib"].gw_actor_act(env.handle, *args), "gw_actor_act")
        return actions_out, probs_out

    def patch_cnn_write_list(self, env, patch: int, out: torch.Tensor, final_out: torch.Tensor | None) -> bool:
        """``env.obs_patch(patch, final=True, out=out, final_out=final_out)`` and, in the same launch,
        the listing of the positions the next ``act_env(..., patch=P, listed=True)`` recomputes
        (gw_patch_cnn_write_list).  False (nothing launched: the caller writes the windows itself)
        while the fused workspace is not derived for the current weights, E % 4 != 0, or a listing
        is still pending (no act since the last one: a second listing would add to its bucket
        counts, which only the act resets)."""
        from . import _lib
        st = self._fast
        if st is None or st["env"] is not env or st.get("patch", 0) != patch or env.E % 4 or st.get("pending"):
            return False
        params = [p for n in self.nets for p in n.parameters()]
        key = (tuple(p._version for p in params), tuple(p.data_ptr() for p in params), getattr(self, "_epoch", 0))
        if st["key"] != key:
            return False
        K, E, P = self.K, env.E, patch
        for t in (out, final_out):
            if t is not None and (t.dtype != torch.float32 or t.numel() != K * E * P * P or not t.is_contiguous()):
                raise ValueError(f"patch_cnn_write_list: need contiguous float32 [K, E, {P}, {P}] buffers")
        with torch.cuda.device(env.device):
            _lib.check(st["lib"].gw_patch_cnn_write_list(env.handle, patch, C.byref(st["spec"]), st["ws"].data_ptr(),
                                                         out.data_ptr(),
                                                         final_out.data_ptr() if final_out is not None else None,
                                                         torch.cuda.current_stream(env.device).cuda_stream),
                       "gw_patch_cnn_write_list")
        st["pending"] = True
        return True

    def _cnn_workspace(self, env, patch: int):
        """The fused CNN path's per-(actors, env) state, its workspace (gw_cnn_prepare /
        gw_patch_cnn_prepare) derived for the current parameters; -> (state, derived now)."""
        from . import _lib
        K, E, dev = self.K, env.E, env.device
        derived = False
        st = self._fast
        if st is None or st["env"] is not env or st.get("patch", 0) != patch:
            if not self.fusable(env, patch):
                raise _lib.GwError("act_env: CNN actor not fusable (needs conv 32-64 k2 s2, hidden 128-128, "
                                   "9 actions, f32, the env's H x W, multiples of 4; or patch=P in 4, 8, 12, 16 "
                                   "with a P x P head)")
            lib = _lib.load()
            ws_n = int(lib.gw_patch_cnn_workspace_floats(patch, env.H, env.W, K, E) if patch
                       else lib.gw_cnn_workspace_floats(env.H, env.W, K, E))
            st = self._fast = dict(env=env, lib=lib, ws=torch.empty(ws_n, dtype=torch.float32, device=dev), key=None,
                                   spec=None, packed=None, patch=patch)
        params = [p for n in self.nets for p in n.parameters()]
        key = (tuple(p._version for p in params), tuple(p.data_ptr() for p in params), getattr(self, "_epoch", 0))
        if key != st["key"]:
            with torch.no_grad():  # the ABI's stacked layouts (include/actor_ops.h gw_cnn_actors)
                pk = dict(
                    conv1_w=torch.stack([n.conv[0].weight for n in self.nets]).contiguous(),
                    conv1_b=torch.stack([n.conv[0].bias for n in self.nets]).contiguous(),
                    conv2_w=torch.stack([n.conv[2].weight for n in self.nets]).contiguous(),
                    conv2_b=torch.stack([n.conv[2].bias for n in self.nets]).contiguous(),
                    lin1_w=torch.stack([n.mlp[0].weight for n in self.nets]).contiguous(),
                    lin1_b=torch.stack([n.mlp[0].bias for n in self.nets]).contiguous(),
                    w2=torch.stack([n.mlp[2].weight.t() for n in self.nets]).contiguous(),
                    b2=torch.stack([n.mlp[2].bias for n in self.nets]).contiguous(),
                    w3=torch.stack([n.mlp[4].weight.t() for n in self.nets]).contiguous(),
                    b3=torch.stack([n.mlp[4].bias for n in self.nets]).contiguous())
            st["packed"] = pk
            st["spec"] = _lib.GwCnnActors(K, self.H, self.W, 32, 64, 128, N_ACTIONS,
                                          *[pk[n].data_ptr() for n in _lib.CNN_PARAM_FIELDS])
            with torch.cuda.device(dev):
                stream = torch.cuda.current_stream(dev).cuda_stream
                if patch:
                    _lib.check(st["lib"].gw_patch_cnn_prepare(env.handle, patch, C.byref(st["spec"]),
                                                              st["ws"].data_ptr(), stream), "gw_patch_cnn_prepare")
                else:
                    _lib.check(st["lib"].gw_cnn_prepare(env.handle, C.byref(st["spec"]), st["ws"].data_ptr(), stream),
                               "gw_cnn_prepare")
            st["key"] = key
            derived = True
        return st, derived

    def _act_env_cnn(self, env, mask, training, tau, seed, counter, uniform, actions_out, probs_out, logits_out,
                     patch=0, counter_dev=None, listed=False):
        """act_env for the CNN head: gw_cnn_act (layer 1 from the obs descriptors through the
        per-position delta table, include/actor_ops.h), then the same fused layers 2-3 + noise +
        softmax + mask + argmax as the MLP path.  patch = P: the head built for P x P inputs on each
        agent's window (gw_patch_cnn_act: per-centre tables + the recomputed positions)."""
        from . import _lib
        K, E, dev = self.K, env.E, env.device
        st, derived = self._cnn_workspace(env, patch)
        if derived:
            listed = False  # a listing made before the workspace was re-derived is not used
        if actions_out is None:
            actions_out = torch.empty((E, K), dtype=torch.int32, device=dev)
        if probs_out is None:
            probs_out = torch.empty((K, E, N_ACTIONS), dtype=torch.float32, device=dev)
        if not (actions_out.dtype == torch.int32 and actions_out.shape == (E, K) and actions_out.is_contiguous()):
            raise ValueError("act_env: actions_out must be a contiguous int32 [E, K] tensor")
        if not (probs_out.dtype == torch.float32 and probs_out.shape == (K, E, N_ACTIONS) and probs_out.is_contiguous()):
            raise ValueError("act_env: probs_out must be a contiguous float32 [K, E, 9] tensor")
        if uniform is not None and not (uniform.dtype == torch.float32 and uniform.shape == (K, E, N_ACTIONS)):
            raise ValueError("act_env: uniform must be float32 [K, E, 9]")
        if mask is not None and not (mask.shape == (E, K) and mask.element_size() == 2 and mask.is_contiguous()):
            raise ValueError("act_env: mask must be a contiguous 16-bit [E, K] tensor")
        args = (C.byref(st["spec"]), st["ws"].data_ptr(), int(bool(training)), float(tau),
                int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF, _ctr_ptr(counter_dev),
                uniform.contiguous().data_ptr() if uniform is not None else None,
                mask.data_ptr() if mask is not None else None, actions_out.data_ptr(), probs_out.data_ptr(),
                logits_out.data_ptr() if logits_out is not None else None, torch.cuda.current_stream(dev).cuda_stream)
        st["pending"] = False  # either act leaves the bucket counters zeroed for the next listing
        if patch and listed:
            _lib.check(st["lib"].gw_patch_cnn_act_listed(env.handle, patch, *args), "gw_patch_cnn_act_listed")
        elif patch:
            _lib.check(st["lib"].gw_patch_cnn_act(env.handle, patch, *args), "gw_patch_cnn_act")
        else:
            _lib.check(st["lib"].gw_cnn_act(env.handle, *args), "gw_cnn_act")
        return actions_out, probs_out
