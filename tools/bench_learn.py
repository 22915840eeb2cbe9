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
    if m.fused:
        # the update alone, as the rollout's learner runs it: critic rows and Gumbel uniforms come
        # with the sample (ReplayRing.sample(critic_in=True, extra_uniform=...)), so no torch
        # cat / rand launches inside the update
        st, ac, rw, ns, dn = batch
        x = m._critic_in(st, ac).contiguous()
        xn = m._critic_in(ns, torch.zeros_like(ac)).contiguous()
        u1 = torch.rand((K, B, 9), device="cuda", generator=g)
        u2 = torch.rand((K, B, 9), device="cuda", generator=g)
        args = (st, ac, rw, ns, dn, u1, u2, (x, xn))
        for _ in range(3):
            m.learn(*args)
        s2 = torch.cuda.Stream()
        s2.wait_stream(torch.cuda.current_stream())
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s2), torch.cuda.graph(g2):
            m.learn(*args)
        torch.cuda.current_stream().wait_stream(s2)
        g2.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            g2.replay()
        torch.cuda.synchronize()
        print(f"batch {B} (fused, rows and uniforms from the sample): graph {(time.perf_counter() - t0) / n * 1e3:.3f} ms/update")


if __name__ == "__main__":
    main()
