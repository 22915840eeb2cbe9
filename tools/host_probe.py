"""Measurement only: host time per C3 step (bench.py's default env loop) split into the return
gather's into() / push() and env.step(), plus the GPU time of the same steps.
Usage: python tools/host_probe.py [steps] [first]  (first: per-step host times of the bench's
timed-region entry)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))

import torch  # noqa: E402

from marlnav.parallel import ReturnGather  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    E = 65536
    env = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=-5.0, max_steps=150, auto_reset=True, seed=42,
                     stats=True)
    env.set_obs_async(True)
    env.reset()
    stats_acc = torch.zeros_like(env.out["stats"])
    gather = ReturnGather(E, 0, 1, env.device)
    ring = [env.out["obs"], torch.empty_like(env.out["obs"])]
    t_into = t_step = t_push = 0.0

    def one(i, timed):
        nonlocal t_into, t_step, t_push
        a = time.perf_counter()
        into = gather.into()
        into["stats_acc"] = stats_acc
        into["obs"] = ring[i % 2]
        b = time.perf_counter()
        env.step(into=into)
        c = time.perf_counter()
        gather.push()
        d = time.perf_counter()
        if timed:
            t_into += b - a
            t_step += c - b
            t_push += d - c

    for i in range(10):
        one(i, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one(i, True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    us = 1e6 / steps
    print(f"host per step: into {t_into * us:.1f} us, env.step {t_step * us:.1f} us, push {t_push * us:.1f} us, "
          f"loop {(t1 - t0) * us:.1f} us; wall per step incl. drain {(t2 - t0) * us:.1f} us")
    env.close()


if __name__ == "__main__" and not (len(sys.argv) > 2 and sys.argv[2] == "first"):
    main()


def first_steps():
    """The bench's timed-region entry (warmup 5, gc, sync, event record) with per-step host times."""
    import gc
    E = 65536
    env = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=-5.0, max_steps=150, auto_reset=True, seed=42,
                     stats=True)
    env.set_obs_async(True)
    env.reset()
    stats_acc = torch.zeros_like(env.out["stats"])
    gather = ReturnGather(E, 0, 1, env.device)
    ring = [env.out["obs"], torch.empty_like(env.out["obs"])]

    parts = []

    def one(i):
        a = time.perf_counter()
        into = gather.into()
        into["stats_acc"] = stats_acc
        into["obs"] = ring[i % 2]
        b = time.perf_counter()
        env.step(into=into)
        c = time.perf_counter()
        gather.push()
        parts.append((round((b - a) * 1e6, 1), round((c - b) * 1e6, 1), round((time.perf_counter() - c) * 1e6, 1)))

    early = bool(os.environ.get("HOST_PROBE_GCEARLY"))  # collect before the last warmup step
    for i in range(5):
        if early and i == 4:
            gc.collect()
            gc.disable()
        one(i)
    stream = torch.cuda.current_stream()
    ev0 = torch.cuda.Event(enable_timing=True)
    if not early:
        gc.collect()
        gc.disable()
    if os.environ.get("HOST_PROBE_SPINSYNC"):  # poll the streams until idle before the sync
        while not stream.query():
            pass
    torch.cuda.synchronize()
    if len(sys.argv) > 3:  # spin the host for argv[3] us after the sync (CPU wake-up hypothesis)
        ts = time.perf_counter()
        while time.perf_counter() - ts < float(sys.argv[3]) * 1e-6:
            pass
    t = [time.perf_counter()]
    ev0.record(stream)
    t.append(time.perf_counter())
    prof = None
    if os.environ.get("HOST_PROBE_PROFILE"):  # cProfile of the first timed step only
        import cProfile
        prof = cProfile.Profile()
    for i in range(5, 25):
        if prof is not None and i == 5:
            prof.enable()
        one(i)
        if prof is not None and i == 5:
            prof.disable()
        t.append(time.perf_counter())
    torch.cuda.synchronize()
    gc.enable()
    d = [round((b - a) * 1e6, 1) for a, b in zip(t, t[1:])]
    print("host us: ev0.record", d[0], "steps", d[1:])
    print("into / env.step / push of the first timed steps:", parts[5:9])
    if prof is not None:
        import pstats
        pstats.Stats(prof).sort_stats("tottime").print_stats(15)
    env.close()


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "first":
    first_steps()
