"""Time one MADDPG update (batch 128, C3 shapes) eager vs HIP-graph replay."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))
import torch  # noqa: E402

from marlnav.maddpg import MADDPG  # noqa: E402


def main():
    K, H, W, B = 2, 32, 32, int(sys.argv[1]) if len(sys.argv) > 1 else 128
    g = torch.Generator(device="cuda").manual_seed(0)
    batch = (torch.randint(-1, 6, (K, B, H, W), device="cuda", generator=g).float(),
             torch.softmax(torch.randn((K, B, 9), device="cuda", generator=g), -1),
             torch.randn((B, K), device="cuda", generator=g, dtype=torch.float64),
             torch.randint(-1, 6, (K, B, H, W), device="cuda", generator=g).float(),
             (torch.rand((B, K), device="cuda", generator=g) < 0.1).to(torch.uint8))
    m = MADDPG(K, H, W, device="cuda", seed=1, capturable=True, batch_size=B)
    if len(sys.argv) > 2:
        m.fused = sys.argv[2] == "fused"
    for _ in range(5):
        m.learn(*batch)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        m.learn(*batch)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / n * 1e3
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(graph):
        m.learn(*batch)
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        graph.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / n * 1e3
    print(f"batch {B} ({'fused' if m.fused else 'autograd'}): eager {eager:.3f} ms/update, graph {gr:.3f} ms/update")


if __name__ == "__main__":
    main()
