"""Time gw_obs_patch alone (HIP events) over E and P: where does the patch writer's time go."""
import os

# the A/B and probe switches exist only in the measurement build (csrc/measure.h)
os.environ.setdefault("MARLNAV_MEASURE", "1")
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "marl-responsible-nav_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import torch  # noqa: E402

from marlnav.vec_env import VecGridEnv  # noqa: E402

CASES = [("grid32", 65536, 11), ("grid32", 16384, 11), ("grid32", 4096, 11), ("grid32", 65536, 3),
         ("grid32", 65536, 16), ("grid32", 65536, 20)]
if len(sys.argv) > 2:
    CASES = [(sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "stamps" else "grid32", int(sys.argv[1]),
              int(sys.argv[2]))]
for scen, E, P in CASES:
    env = VecGridEnv(scen, num_envs=E, fear=False, seed=1, obs=False)
    env.reset()
    env.step()
    out = torch.empty((env.K, E, P, P), device="cuda")
    for _ in range(3):
        env.obs_patch(P, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        env.obs_patch(P, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    gb = env.K * E * P * P * 4 / 1e9
    print(f"{scen} E={E} P={P}: {us:.1f} us per launch, {gb * 1e3:.1f} MB, {gb / (us * 1e-6):.0f} GB/s", flush=True)
    env.close()

# per-block wall-clock stamps (100 MHz) of one launch: how many blocks overlap, where a block's
# time goes (entry -> staged -> windows assembled -> stored)
if "stamps" in sys.argv[3:]:
    import ctypes as C
    import numpy as np
    from marlnav import _lib
    lib = _lib.load()
    lib.gw_patch_debug_buffer.argtypes = [C.c_void_p]
    E, P = int(sys.argv[1]), int(sys.argv[2])
    scen = sys.argv[3] if sys.argv[3] != "stamps" else "grid32"
    env = VecGridEnv(scen, num_envs=E, fear=False, seed=1, obs=False)
    env.reset()
    env.step()
    out = torch.empty((env.K, E, P, P), device="cuda")
    nb = (E + 31) // 32
    dbg = torch.zeros((nb, 4), dtype=torch.int64, device="cuda")
    env.obs_patch(P, out=out)
    lib.gw_patch_debug_buffer(dbg.data_ptr())
    env.obs_patch(P, out=out)
    torch.cuda.synchronize()
    lib.gw_patch_debug_buffer(None)
    d = dbg.cpu().numpy().astype(np.float64)
    d[:, 2] = np.where(d[:, 2] == 0, d[:, 1], d[:, 2])  # MODE 2 / 3 assemble nothing in LDS
    d -= d[:, 0].min()
    us = d / 100.0
    print(f"blocks {nb}: kernel span {us[:, 3].max():.1f} us; block lifetime mean {np.mean(us[:, 3] - us[:, 0]):.2f} us "
          f"(staging {np.mean(us[:, 1] - us[:, 0]):.2f}, windows {np.mean(us[:, 2] - us[:, 1]):.2f}, "
          f"store {np.mean(us[:, 3] - us[:, 2]):.2f}); block start times: first {us[:, 0].min():.2f} "
          f"median {np.median(us[:, 0]):.2f} last {us[:, 0].max():.2f} us")
    ts = np.linspace(0, us[:, 3].max(), 12)
    conc = [int(((us[:, 0] <= t) & (us[:, 3] >= t)).sum()) for t in ts]
    print("resident blocks over time:", conc)
