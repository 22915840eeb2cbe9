"""gw_return_compact (include/rollout_ops.h) == ReturnGather's torch compaction.

The reference appends ``scores[i]`` to ``completed_episode_scores`` for every env done this
step (maddpg/agent.py:229-247).  ReturnGather keeps that list on the device; on the GPU its
window of gathered steps is compacted by two HIP launches.  Checked here against the torch-op
compaction (the CPU / gloo path) on synthetic windows: several ranks with padded slots, ragged
shards, empty windows, dense and sparse done patterns, ring wrap-around and windows holding
more completions than the ring.  Bit-exact (a scatter of f64 values)."""
import ctypes as C

import numpy as np
import pytest
import torch

from marlnav import _lib
from marlnav.parallel import ReturnGather

pytestmark = pytest.mark.gpu


def _hip_and_torch(world, emax, counts, steps, capacity, density, seed, windows=3):
    g = torch.Generator().manual_seed(seed)
    G = sum(counts)
    out = []  # two rings fed the same windows: HIP (cuda) and torch ops (cpu)
    for dev in ("cuda", "cpu"):
        rg = ReturnGather.__new__(ReturnGather)
        rg.world, rg.emax, rg.G = world, emax, G
        rg.distributed = False  # the full-slot format (one rank's path), fed `world` ranks' slots
        rg.slot_bytes = 8 * emax + (-(-emax // 8)) * 8
        rg.window, rg.capacity, rg.device = steps, capacity, torch.device(dev)
        rg._recv = torch.zeros((steps, world, rg.slot_bytes), dtype=torch.uint8, device=dev)
        rg.scores = torch.zeros(capacity + 1, dtype=torch.float64, device=dev)
        rg.n_completed = torch.zeros((), dtype=torch.int64, device=dev)
        rg._work, rg._fill, rg._scratch = [None, None], 0, None
        out.append(rg)
    for w in range(windows):
        T = steps if w != 1 else max(1, steps // 3)  # a short window too
        rets = torch.randn((T, world, emax), generator=g, dtype=torch.float64)
        done = (torch.rand((T, world, emax), generator=g) < density).to(torch.uint8)
        for r in range(world):  # padding past each rank's shard is never done
            done[:, r, counts[r]:] = 0
        slot = torch.zeros((T, world, out[0].slot_bytes), dtype=torch.uint8)
        slot[:, :, : 8 * emax] = rets.view(torch.uint8).reshape(T, world, 8 * emax)
        slot[:, :, 8 * emax: 9 * emax] = done
        for rg in out:
            rg._recv[:T].copy_(slot.to(rg.device))
            rg._fill = T
            rg.compact()
    torch.cuda.synchronize()
    hip, ref = out
    assert int(hip.n_completed) == int(ref.n_completed)
    np.testing.assert_array_equal(hip.scores[:capacity].cpu().numpy(), ref.scores[:capacity].numpy())
    np.testing.assert_array_equal(hip.completed(), ref.completed())
    return int(ref.n_completed)


@pytest.mark.parametrize("world,emax,counts,steps,capacity,density", [
    (1, 4096, [4096], 16, 1 << 20, 0.05),          # one rank, sparse, no wrap
    (3, 1367, [1367, 1367, 1366], 7, 500, 0.3),    # ragged shards, ring wraps every window
    (2, 33, [33, 31], 5, 10_000, 1.0),             # every element done
    (8, 8192, [8192] * 8, 4, 3000, 0.02),          # more completions per window than the ring
    (2, 100, [100, 100], 3, 64, 0.0),              # no completions at all
])
def test_compaction_matches_torch(world, emax, counts, steps, capacity, density):
    n = _hip_and_torch(world, emax, counts, steps, capacity, density, seed=world * 7 + emax)
    if density > 0:
        assert n > 0


def test_bad_arguments_rejected():
    lib = _lib.load()
    st = lib.gw_return_compact(None, 1, 1, 16, 8 * 16, None, 10, None, None, C.c_void_p(0))
    assert st != 0 and b"bad argument" in lib.gw_last_error()
