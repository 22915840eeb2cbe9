"""The packed multi-rank return gather's kernels (gw_gather_pack / gw_gather_unpack,
include/rollout_ops.h) on one GPU, world simulated: R "ranks" pack their steps, the slots are
laid out as all_gather_into_tensor lays them ([step][rank][slot]), every window is unpacked.

The completed-episode list (maddpg/agent.py:229-247: per step, the done envs' returns by global
env id; rank-major contiguous shards) must come out bit for bit, also when `cap` is far below
the completions per step (backlogs drained over later steps, steps emitted late), with ragged
shards, and with a score ring smaller than the list (the last `capacity` kept)."""
import ctypes as C

import numpy as np
import pytest
import torch

from marlnav import _lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,shards,cap,window,capacity", [(2, (513, 512), 16, 5, 1 << 16), (3, (100, 99, 99), 64, 4, 1 << 16),
                                                           (2, (300, 300), 7, 3, 97)])
def test_pack_unpack_reference_order(R, shards, cap, window, capacity):
    lib = _lib.load()
    dev = "cuda"
    steps = 23
    rng = np.random.default_rng(1)
    emax = max(shards)
    fifo_cap = 2 * window * emax + emax
    slot_bytes = 32 + 8 * cap
    pend_cap = 512  # steps waiting for a backlog (no cap adaptation here, unlike ReturnGather)
    s = torch.cuda.current_stream().cuda_stream
    fifo = [torch.zeros(fifo_cap, dtype=torch.float64, device=dev) for _ in range(R)]
    ctl = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(R)]
    scratch = [torch.zeros(int(lib.gw_gather_pack_scratch(n)), dtype=torch.int32, device=dev) for n in shards]
    recv = torch.zeros((window, R, slot_bytes), dtype=torch.uint8, device=dev)
    mirror = torch.zeros((R, fifo_cap), dtype=torch.float64, device=dev)
    rst = torch.zeros(2 * R + 4, dtype=torch.int64, device=dev)
    pend = torch.zeros((pend_cap, R), dtype=torch.int32, device=dev)
    plan_cap = int(lib.gw_gather_unpack_plan_cap(window, R, pend_cap))
    plan = torch.zeros(plan_cap * 40 + 32, dtype=torch.uint8, device=dev)
    scores = torch.zeros(capacity + 1, dtype=torch.float64, device=dev)
    n_completed = torch.zeros((), dtype=torch.int64, device=dev)
    want = []
    fill = 0

    def unpack(n):
        _lib.check(lib.gw_gather_unpack(recv.data_ptr(), n, R, slot_bytes, mirror.data_ptr(), fifo_cap, rst.data_ptr(),
                                        pend.data_ptr(), pend_cap, plan.data_ptr(), plan_cap, scores.data_ptr(),
                                        capacity, n_completed.data_ptr(), C.c_void_p(s)), "gw_gather_unpack")

    for t in range(steps):
        for r, n in enumerate(shards):
            ret = torch.tensor(rng.normal(size=n), device=dev)
            done = torch.tensor(rng.random(n) < 0.3, dtype=torch.uint8, device=dev)
            want.extend(ret[done.bool()].tolist())
            _lib.check(lib.gw_gather_pack(ret.data_ptr(), done.data_ptr(), n, cap, fifo[r].data_ptr(), fifo_cap,
                                          ctl[r].data_ptr(), scratch[r].data_ptr(), recv[fill, r].data_ptr(),
                                          C.c_void_p(s)), "gw_gather_pack")
        fill += 1
        if fill == window:
            unpack(fill)
            fill = 0
    # drain: steps with empty sends until every backlog has gone out
    for t in range(400):
        for r, n in enumerate(shards):
            z = torch.zeros(n, dtype=torch.float64, device=dev)
            _lib.check(lib.gw_gather_pack(z.data_ptr(), torch.zeros(n, dtype=torch.uint8, device=dev).data_ptr(), n,
                                          cap, fifo[r].data_ptr(), fifo_cap, ctl[r].data_ptr(), scratch[r].data_ptr(),
                                          recv[fill, r].data_ptr(), C.c_void_p(s)), "gw_gather_pack")
        fill += 1
        if fill == window:
            unpack(fill)
            fill = 0
    if fill:
        unpack(fill)
    torch.cuda.synchronize()
    assert int(rst[2 * R + 2]) == 0, "overflow flagged"
    n = int(n_completed)
    assert n == len(want)
    m = min(n, capacity)
    got = scores[(torch.arange(m, device=dev) + (n - m)) % capacity].cpu().numpy()
    np.testing.assert_array_equal(got, np.array(want[-m:]))
    # the headers: the backlog was exercised when cap is small
    assert all(int(c[0]) == int(c[1]) for c in ctl)  # every FIFO drained (head == tail)
