"""The fused update's weights after a few updates on a fixed batch, saved for a bit-for-bit
comparison across builds / switches (e.g. GW_TAIL_PAR=0 vs the three-group critic tail).
    python tools/tail_ab.py out.safetensors [updates]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))
import torch  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

from marlnav.maddpg import MADDPG  # noqa: E402


def main():
    K, H, W, B = 2, 32, 32, 128
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    g = torch.Generator(device="cuda").manual_seed(0)
    batch = (torch.randint(-1, 6, (K, B, H, W), device="cuda", generator=g).float(),
             torch.softmax(torch.randn((K, B, 9), device="cuda", generator=g), -1),
             torch.randn((B, K), device="cuda", generator=g, dtype=torch.float64),
             torch.randint(-1, 6, (K, B, H, W), device="cuda", generator=g).float(),
             (torch.rand((B, K), device="cuda", generator=g) < 0.1).to(torch.uint8),
             torch.rand((K, B, 9), device="cuda", generator=g),
             torch.rand((K, B, 9), device="cuda", generator=g))
    m = MADDPG(K, H, W, device="cuda", seed=1, batch_size=B)
    assert m.fused
    for _ in range(n):
        m.learn(*batch)
    torch.cuda.synchronize()
    save_file({k: v.detach().cpu().contiguous() for k, v in m.state_dict().items()}, sys.argv[1])
    print("saved", len(m.state_dict()), "tensors after", n, "updates")


if __name__ == "__main__":
    main()
