"""The stacked MLPs' hidden-layer epilogue as one HIP launch (gw_ln_relu_fwd / gw_ln_relu_bwd,
marlnav/actor.py ln_relu) == torch's F.layer_norm + addcmul + relu (the agilerl EvolvableMLP
layer: Linear -> LayerNorm -> ReLU, maddpg/agent.py:41-65 networks) in fp32, forward and
backward (input gradient and the LayerNorm affine gradients, which the kernel adds into the
parameters' existing .grad as autograd accumulates).
Tolerance: 2e-5 relative / 2e-6 absolute on y and dz (the row mean / variance are summed in a
different order than torch's Welford), 1e-4 relative on the affine gradients (sums over R rows)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _torch_ref(z, w, b):
    return F.relu(torch.addcmul(b, F.layer_norm(z, (z.shape[-1],)), w))


@pytest.mark.parametrize("K,R,h", [(2, 128, 128), (3, 37, 100), (1, 5, 512), (2, 4096, 64)])
def test_ln_relu_matches_torch(K, R, h):
    from marlnav.actor import ln_relu
    g = torch.Generator(device="cuda").manual_seed(K * 1000 + h)
    z0 = torch.randn((K, R, h), device="cuda", generator=g) * 3 + 0.5
    w0 = torch.randn((K, 1, h), device="cuda", generator=g)
    b0 = torch.randn((K, 1, h), device="cuda", generator=g) * 0.3
    dy = torch.randn((K, R, h), device="cuda", generator=g)
    pre_w = torch.randn((K, 1, h), device="cuda", generator=g)  # an existing .grad to accumulate into
    pre_b = torch.randn((K, 1, h), device="cuda", generator=g)

    zr, wr, br = (t.clone().requires_grad_(True) for t in (z0, w0, b0))
    yr = _torch_ref(zr, wr, br)
    wr.grad, br.grad = pre_w.clone(), pre_b.clone()
    yr.backward(dy)

    z, w, b = (t.clone().requires_grad_(True) for t in (z0, w0, b0))
    w.grad, b.grad = pre_w.clone(), pre_b.clone()
    y = ln_relu(z, w, b)
    torch.testing.assert_close(y, yr.detach(), rtol=2e-5, atol=2e-6)
    y.backward(dy)
    torch.testing.assert_close(z.grad, zr.grad, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(b.grad, br.grad, rtol=1e-4, atol=1e-4)


def test_ln_relu_no_grad_and_fresh_grad():
    """Under no_grad nothing is saved; a parameter without a .grad gets one through autograd."""
    from marlnav.actor import ln_relu
    g = torch.Generator(device="cuda").manual_seed(7)
    z = torch.randn((2, 64, 128), device="cuda", generator=g)
    w = torch.randn((2, 1, 128), device="cuda", generator=g)
    b = torch.randn((2, 1, 128), device="cuda", generator=g)
    with torch.no_grad():
        torch.testing.assert_close(ln_relu(z, w, b), _torch_ref(z, w, b), rtol=2e-5, atol=2e-6)
    wp, bp = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ln_relu(z, wp, bp).sum().backward()
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    _torch_ref(z, wr, br).sum().backward()
    torch.testing.assert_close(wp.grad, wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bp.grad, br.grad, rtol=1e-4, atol=1e-4)


def test_stacked_mlp_takes_the_hip_epilogue():
    """StackedMLPActors on the GPU with GW_LN_FUSED=1 runs ln_relu and matches the torch
    composition it replaces."""
    from marlnav import actor
    net = actor.StackedMLPActors(2, 1024, (128, 128), device="cuda", seed=4)
    x = torch.randn((2, 128, 1024), device="cuda")
    fused = actor._FUSED_LN
    try:
        actor._FUSED_LN = True  # GW_LN_FUSED=1
        assert actor._fused_ln_ok(torch.empty((2, 1, 128), device="cuda"))
        y = net(x)
        actor._FUSED_LN = False
        y_ref = net(x)
    finally:
        actor._FUSED_LN = fused
    torch.testing.assert_close(y, y_ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("rows,n", [(256, 9), (1000, 9), (3, 5)])
def test_gumbel_softmax_hip_matches_torch(rows, n):
    """gw_gumbel_softmax (the no-gradient GumbelSoftmax of MADDPG.learn's target actions) == the
    torch composition softmax((logits - log(-log(u + eps) + eps)) / tau).  Tolerance 2e-6 abs
    (logf / expf ulps and the softmax sum order)."""
    from marlnav.maddpg import _gumbel_hip, gumbel_softmax
    g = torch.Generator(device="cuda").manual_seed(rows + n)
    logits = torch.randn((rows, n), device="cuda", generator=g) * 4
    u = torch.rand((rows, n), device="cuda", generator=g)
    u[0, 0] = 0.0  # the eps guards
    got = _gumbel_hip(logits, u, tau=0.7)
    want = torch.softmax((logits - torch.log(-torch.log(u + 1e-20) + 1e-20)) / 0.7, dim=-1)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=2e-6)
    with torch.no_grad():  # the public helper is the torch formula itself, gradient or not
        assert torch.equal(gumbel_softmax(logits, u, tau=0.7), want)
    lg = logits.clone().requires_grad_(True)
    gumbel_softmax(lg, u, tau=0.7).sum().backward()
    assert lg.grad is not None


@pytest.mark.parametrize("K,R,h", [(2, 128, 128), (3, 37, 100), (1, 5, 200)])
def test_affine_relu_matches_torch(K, R, h):
    """gw_affine_relu_fwd / _bwd (the default learner epilogue after torch's F.layer_norm) ==
    addcmul + relu: the forward bit for bit; the input gradient bit for bit; the affine
    gradients (row sums in another order) within 1e-5 relative."""
    from marlnav.actor import affine_relu
    g = torch.Generator(device="cuda").manual_seed(K * 7 + h)
    xh0 = torch.randn((K, R, h), device="cuda", generator=g)
    w0 = torch.randn((K, 1, h), device="cuda", generator=g)
    b0 = torch.randn((K, 1, h), device="cuda", generator=g) * 0.3
    dy = torch.randn((K, R, h), device="cuda", generator=g)
    pre_w = torch.randn((K, 1, h), device="cuda", generator=g)
    pre_b = torch.randn((K, 1, h), device="cuda", generator=g)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (xh0, w0, b0))
    yr = torch.relu(torch.addcmul(br, xr, wr))
    wr.grad, br.grad = pre_w.clone(), pre_b.clone()
    yr.backward(dy)
    x, w, b = (t.clone().requires_grad_(True) for t in (xh0, w0, b0))
    w.grad, b.grad = pre_w.clone(), pre_b.clone()
    y = affine_relu(x, w, b)
    # torch's addcmul on ROCm rounds the product, then the sum (no fma contraction): measured
    assert torch.equal(yr.detach(), torch.relu(xh0 * w0 + b0))
    assert torch.equal(y, yr.detach())
    y.backward(dy)
    assert torch.equal(x.grad, xr.grad)
    torch.testing.assert_close(w.grad, wr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(b.grad, br.grad, rtol=1e-5, atol=1e-5)
