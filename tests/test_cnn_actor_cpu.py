"""CNN actor head (configs/cnn.yaml: conv 32-64, k2 s2, 128-128): the per-patch GEMM form used for
kernel == stride convs equals the nn.Conv2d form (CPU, float32)."""
import pytest
import torch

from marlnav.actor import CNNActor


@pytest.mark.parametrize("H,W", [(64, 64), (32, 32), (10, 16), (16, 12)])
def test_patch_gemm_matches_conv(H, W):
    torch.manual_seed(H * 100 + W)
    m = CNNActor(H, W)
    x = torch.randint(-1, 14, (5, 1, H, W)).float()
    x[0, 0, 0, 0] = 0.5
    ref = m.mlp(m.conv(x).flatten(1))
    torch.testing.assert_close(m(x), ref, rtol=1e-5, atol=1e-5)
    assert m.patchify == (H % 4 == 0 and W % 4 == 0)
