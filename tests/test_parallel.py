"""Multi-process (world_size 2, gloo on CPU) checks of the sharding + reduction logic.

The GPU run uses the same code with the nccl (RCCL) backend: marlnav.parallel.shard gives each
rank a contiguous range of global env ids, every draw is keyed by the global id, and the
per-step StatsReducer all-reduces the step's partial sums.  Here the per-env step is the C
oracle (same spec as the kernels, pinned bit-exact to them by tests/test_gpu_parity.py).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from marlnav.parallel import StatsReducer, shard

STATS = 8


@pytest.mark.parametrize("G,world", [(1, 1), (7, 2), (65536, 8), (524288, 8), (10, 3), (5, 8)])
def test_shard_partitions_exactly(G, world):
    seen = []
    for r in range(world):
        off, cnt = shard(G, r, world)
        seen.extend(range(off, off + cnt))
    assert seen == list(range(G))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _per_env_stats(outs, E):
    """The step kernel's stats fields, per env, from oracle outputs."""
    st = np.zeros((E, STATS))
    for e in range(E):
        o = outs[e]
        done = bool(o.done)
        st[e] = [o.ep_return if done else 0.0, float(done), o.fear[0] + o.fear[1], o.crashes, o.apples_caught,
                 o.shaped[0] + o.shaped[1], o.ep_len if done else 0.0, 1.0]
    return st


def _worker(rank, world, port, G, steps, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from marlnav import scenario as S
    from oracle import oracle as O
    sc = S.builtin("grid32")
    off, cnt = shard(G, rank, world)
    orc = O.OracleEnvs(sc, cnt, fear=True, seed=5, env_offset=off)
    outs = (O.StepOut * cnt)()
    red = StatsReducer(STATS, "cpu")
    rets = []
    for _ in range(steps):
        orc.vec_step(None, outs=outs, nthreads=1)
        partial = torch.tensor(_per_env_stats(outs, cnt))
        red.push(partial)  # async all-reduce, double-buffered
        rets.append([outs[e].ep_return for e in range(cnt)])
    totals = red.result().numpy()
    pos = torch.tensor(orc.positions())
    gathered = [torch.zeros((shard(G, r, world)[1], sc.N), dtype=pos.dtype) for r in range(world)]
    dist.all_gather(gathered, pos) if all(g.shape == pos.shape for g in gathered) else None
    if rank == 0:
        np.save(os.path.join(outdir, "totals.npy"), totals)
        np.save(os.path.join(outdir, "pos.npy"), torch.cat(gathered).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_matches_single_process():
    G, steps, world = 512, 15, 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), G, steps, d), nprocs=world, join=True)
        totals = np.load(os.path.join(d, "totals.npy"))
        pos = np.load(os.path.join(d, "pos.npy"))
    from marlnav import scenario as S
    from oracle import oracle as O
    sc = S.builtin("grid32")
    orc = O.OracleEnvs(sc, G, fear=True, seed=5)
    outs = (O.StepOut * G)()
    ref = np.zeros(STATS)
    for _ in range(steps):
        orc.vec_step(None, outs=outs, nthreads=4)
        ref += _per_env_stats(outs, G).sum(0)
    np.testing.assert_array_equal(pos, orc.positions())       # sharded trajectories == single run
    np.testing.assert_allclose(totals, ref, rtol=1e-12)        # reduced statistics == single run
    assert ref[1] > 0                                          # some episodes completed
