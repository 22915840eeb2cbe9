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

from marlnav.parallel import ReturnGather, StatsReducer, shard

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
    gat = ReturnGather(G, rank, world, "cpu", window=4)          # wraps the receive ring 3x
    gat_small = ReturnGather(G, rank, world, "cpu", window=5, capacity=37)  # keeps the last 37
    # a cap far below the completions per step: backlogs, late steps, the cap doubling per window
    gat_tiny = ReturnGather(G, rank, world, "cpu", window=3, cap=2)
    caps = []
    for _ in range(steps):
        orc.vec_step(None, outs=outs, nthreads=1)
        partial = torch.tensor(_per_env_stats(outs, cnt))
        red.push(partial)  # async all-reduce, double-buffered
        ret = torch.tensor([outs[e].ep_return for e in range(cnt)], dtype=torch.float64)
        done = torch.tensor([outs[e].done for e in range(cnt)], dtype=torch.uint8)
        gat.push(ret, done)          # copy path
        into = gat_small.into()      # zero-copy path: the "step" writes the send buffer
        into["ep_return"].copy_(ret)
        into["done"].copy_(done)
        gat_small.push()
        gat_tiny.push(ret, done)
        caps.append(gat_tiny.cap)
    totals = red.result().numpy()
    np.save(os.path.join(outdir, f"completed{rank}.npy"), gat.completed())
    np.save(os.path.join(outdir, f"completed_small{rank}.npy"), gat_small.completed())
    np.save(os.path.join(outdir, f"completed_tiny{rank}.npy"), gat_tiny.completed())
    np.save(os.path.join(outdir, f"caps{rank}.npy"), np.array(caps))
    # the per-step message: a header and cap returns, not 9 bytes per env
    assert gat.slot_bytes == 32 + 8 * gat.cap < 9 * gat.emax
    emax = -(-G // world)
    pos = torch.zeros((emax, sc.N), dtype=torch.int32)
    pos[:cnt] = torch.tensor(orc.positions(), dtype=torch.int32)
    gathered = [torch.zeros_like(pos) for _ in range(world)]
    dist.all_gather(gathered, pos)
    if rank == 0:
        np.save(os.path.join(outdir, "totals.npy"), totals)
        np.save(os.path.join(outdir, "pos.npy"),
                torch.cat([g[: shard(G, r, world)[1]] for r, g in enumerate(gathered)]).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("G", [512, 513])
def test_gloo_world2_matches_single_process(G):
    """Sharded over 2 gloo ranks (513: ragged shards, the gather pads the shorter one) ==
    one process: positions, the all-reduced statistics, and the all-gathered completed-episode
    returns (every rank gets the global list, in the reference's order: step, then env id)."""
    steps, world = 15, 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), G, steps, d), nprocs=world, join=True)
        totals = np.load(os.path.join(d, "totals.npy"))
        pos = np.load(os.path.join(d, "pos.npy"))
        completed = [np.load(os.path.join(d, f"completed{r}.npy")) for r in range(world)]
        completed_small = [np.load(os.path.join(d, f"completed_small{r}.npy")) for r in range(world)]
        completed_tiny = [np.load(os.path.join(d, f"completed_tiny{r}.npy")) for r in range(world)]
        caps = [np.load(os.path.join(d, f"caps{r}.npy")) for r in range(world)]
    from marlnav import scenario as S
    from oracle import oracle as O
    sc = S.builtin("grid32")
    orc = O.OracleEnvs(sc, G, fear=True, seed=5)
    outs = (O.StepOut * G)()
    ref = np.zeros(STATS)
    scores = []  # maddpg/agent.py:229-247: completed_episode_scores.append(scores[i]) per done env
    for _ in range(steps):
        orc.vec_step(None, outs=outs, nthreads=4)
        ref += _per_env_stats(outs, G).sum(0)
        scores.extend(outs[e].ep_return for e in range(G) if outs[e].done)
    scores = np.array(scores)
    for r in range(world):
        np.testing.assert_array_equal(completed[r], scores)
        np.testing.assert_array_equal(completed_small[r], scores[-37:])
        np.testing.assert_array_equal(completed_tiny[r], scores)
    np.testing.assert_array_equal(caps[0], caps[1])             # every rank adapts alike
    assert caps[0][0] == 2 and caps[0][-1] > 2                  # ... and the cap grew
    assert len(scores) > 37                                    # the small ring wrapped
    np.testing.assert_array_equal(pos, orc.positions())       # sharded trajectories == single run
    np.testing.assert_allclose(totals, ref, rtol=1e-12)        # reduced statistics == single run
    assert ref[1] > 0                                          # some episodes completed


def _burst_series(G, steps, seed=3):
    """Synthetic per-step (returns [G] f64, done [G] u8) of G global envs: a low completion rate,
    a burst where every env ends at once (step 4: episodes that started together), and a final
    step where every env ends (the run stops right after a burst)."""
    rng = np.random.default_rng(seed)
    out = []
    for t in range(steps):
        ret = rng.normal(size=G)
        done = rng.random(G) < 0.03
        if t == 4 or t == steps - 1:
            done[:] = True
        out.append((ret, done.astype(np.uint8)))
    return out


def _gather_worker(rank, world, port, G, steps, outdir, mid_window_reader):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = shard(G, rank, world)
    gat = ReturnGather(G, rank, world, "cpu", window=4, cap=3)  # cap far below the bursts
    caps, mid = [], None
    for t, (ret, done) in enumerate(_burst_series(G, steps)):
        gat.push(torch.from_numpy(ret[off: off + cnt]), torch.from_numpy(done[off: off + cnt]))
        caps.append(gat.cap)
        if rank == 0 and mid_window_reader and t in (5, 9, 10):
            # rank-0-only logging mid-window: compacts on this rank alone
            mid = gat.completed()
    added = gat.drain()  # collective: every rank, same point
    np.save(os.path.join(outdir, f"done{rank}.npy"), gat.completed())
    np.save(os.path.join(outdir, f"caps{rank}.npy"), np.array(caps + [gat.cap]))
    np.save(os.path.join(outdir, f"added{rank}.npy"), np.array([added, gat.slot_bytes]))
    if mid is not None:
        np.save(os.path.join(outdir, "mid.npy"), mid)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,G,reader", [(4, 203, False), (4, 203, True), (2, 64, True)])
def test_gloo_return_gather_bursts_match_single_process(world, G, reader):
    """world 4 (203 envs: ragged shards 51/51/51/50) and 2: completion bursts far above ``cap``
    (3) force backlogs and cap doubling, the run ends right after a burst, and (reader) rank 0
    alone calls completed() mid-window.  After the collective drain() every rank holds the one-
    process list (step, then global env id) bit for bit, and every rank resized its slots at the
    same steps."""
    steps = 13
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gather_worker, args=(world, _free_port(), G, steps, d, reader), nprocs=world, join=True)
        got = [np.load(os.path.join(d, f"done{r}.npy")) for r in range(world)]
        caps = [np.load(os.path.join(d, f"caps{r}.npy")) for r in range(world)]
        added = [np.load(os.path.join(d, f"added{r}.npy")) for r in range(world)]
        mid = np.load(os.path.join(d, "mid.npy")) if reader else None
    want = np.concatenate([ret[done != 0] for ret, done in _burst_series(G, steps)])
    for r in range(world):
        np.testing.assert_array_equal(got[r], want)
        np.testing.assert_array_equal(caps[r], caps[0])
        np.testing.assert_array_equal(added[r], added[0])
    assert caps[0][0] == 3 and caps[0][-1] > 3       # the bursts grew the cap
    assert added[0][0] > 0                           # the final burst needed the drain
    if reader:  # a mid-window read is a prefix of the full list
        np.testing.assert_array_equal(mid, want[: len(mid)])


def test_return_gather_single_process_order_and_rings():
    """World size 1 (no process group): the compacted list == the per-step done envs' returns in
    env order, across receive-ring wraps (window 3) and a score ring smaller than the total."""
    rng = np.random.default_rng(0)
    E, steps = 50, 20
    big = ReturnGather(E, 0, 1, "cpu", window=3)
    small = ReturnGather(E, 0, 1, "cpu", window=7, capacity=13)
    want = []
    for t in range(steps):
        ret = torch.tensor(rng.normal(size=E))
        done = torch.tensor(rng.random(E) < 0.2, dtype=torch.uint8)
        want.extend(ret[done.bool()].tolist())
        big.push(ret, done)
        small.push(ret, done)
        if t == 10:  # a mid-window read compacts early; later steps continue the list
            np.testing.assert_array_equal(big.completed(), np.array(want))
    np.testing.assert_array_equal(big.completed(), np.array(want))
    np.testing.assert_array_equal(small.completed(), np.array(want[-13:]))
    np.testing.assert_array_equal(big.completed(last=5), np.array(want[-5:]))
    assert int(big.n_completed) == len(want) > 13


def test_cap_doubles_after_a_window_with_a_backlog():
    """ReturnGather._adapt_from: any backlog in the window before doubles ``cap`` (every rank
    reads the same headers, so this is the whole decision); a window without one keeps it."""
    def run(maxbs):
        g = ReturnGather.__new__(ReturnGather)
        g.cap, g.emax, g.fifo_cap = 64, 200, 2 * 64 * 200 + 200
        g._maxb_host = torch.zeros(2, dtype=torch.int64)
        g._alloc_slots = lambda: None
        caps = []
        for w, mb in enumerate(maxbs):
            g._maxb_host[w % 2] = mb
            g._nwin = w + 2
            g._adapt_from(None)
            caps.append(g.cap)
        return caps

    assert run([0, 5, 0, 900, 1]) == [64, 128, 128, 200, 200]  # capped at the shard
