"""Measurement only: phase durations of step_v2_block (thread 0 of each block) at C2's shape, from
the GW_STEP_CLK build (tools/step_clk.sh; loaded through MARLNAV_LIB, never by the product path).

Slots: 0 entry, 1 after the state loads + LDS table fill + barrier, 2 after the action draws,
3 after the world update, 4 after finish_env (rewards, resets, outputs, descriptor), 5 before the
block statistics, 6 after them.  Cycles are s_memtime ticks (shader clock).
Usage: MARLNAV_LIB=.../libgridenv_clk.so python tools/step_clk.py [envs] [steps] [merged|sync|noobs] [scenario] [envs per block]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "marl-responsible-nav_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlnav import _lib  # noqa: E402
from marlnav import scenario as S  # noqa: E402
from marlnav.vec_env import VecGridEnv  # noqa: E402


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    mode = sys.argv[3] if len(sys.argv) > 3 else "merged"   # merged | sync | noobs
    scen = sys.argv[4] if len(sys.argv) > 4 else "grid32"
    assert os.environ.get("MARLNAV_LIB"), "needs the measurement build (tools/step_clk.sh)"
    lib = _lib.load()
    lib.gw_step_debug_clocks.argtypes = [C.c_void_p]
    env = VecGridEnv(S.builtin(scen), num_envs=E, fear=False, seed=3, obs=mode != "noobs")
    if mode == "merged":
        env.set_obs_async(True)
    env.reset()
    for _ in range(steps):
        env.step()
    torch.cuda.synchronize()
    print("kernel path:", getattr(env, "kernel_path", "?"))
    buf = np.zeros((64, 16), dtype=np.uint64)
    assert lib.gw_step_debug_clocks(buf.ctypes.data) == 0
    be = int(sys.argv[5]) if len(sys.argv) > 5 else 32  # envs per step_v2 block (128 for N > 4)
    nb = min(64, (E + be - 1) // be)
    d = buf[:nb, :7].astype(np.int64)
    ph = np.diff(d, axis=1)
    names = ["loads+fill+sync", "actions", "world update", "finish_env", "to stats", "block stats"]
    print(f"{nb} blocks, cycles per phase (median / max over blocks), ~us at 2.4 GHz:")
    for i, n in enumerate(names):
        print(f"  {n:16s} {int(np.median(ph[:, i])):7d} {int(ph[:, i].max()):7d}  {np.median(ph[:, i]) / 2400:6.2f}")
    tot = d[:, 6] - d[:, 0]
    print(f"  {'total':16s} {int(np.median(tot)):7d} {int(tot.max()):7d}  {np.median(tot) / 2400:6.2f}")
    env.close()


if __name__ == "__main__":
    main()
