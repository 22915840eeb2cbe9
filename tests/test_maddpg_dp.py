"""Data-parallel MADDPG learner (reference learn call site
maddpg/agent.py:199-224): 2 ranks, each learning on its half of a batch, == one process learning
on the whole batch, and the two replicas stay identical.

Per rank: the networks are broadcast from rank 0 at construction (rank 1 is built with another
seed, so the broadcast is what makes them equal), each backward is followed by one all-reduce
of the flat gradient buffer averaged over the ranks.  With equal half-batches the averaged
gradient is that of the mean loss over the concatenated batch; only the summation order
differs, so the tolerance is test_maddpg.py's GPU one: every parameter tensor within 1e-4
relative L2 and 2 * lr * updates elementwise (Adam's normalised step turns rounding-level
gradient differences into steps of up to lr).  The replicas are compared bit for bit.

CPU: gloo, world size 2, the learner's torch path.  GPU (marked): gloo on CUDA tensors, 2 ranks
on one MI355X (RCCL refuses two ranks on one device), the HIP flat path, eager and as the
three captured graph segments with the all-reduces between them.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

K, H, W, B, UPDATES, LR = 2, 6, 5, 32, 4, 1e-2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(device, B_=B, H_=H, W_=W):
    g = torch.Generator(device=device).manual_seed(11)
    out = []
    for _ in range(UPDATES):
        out.append(dict(
            states=torch.randint(-1, 6, (K, B_, H_, W_), generator=g, device=device).float(),
            next_states=torch.randint(-1, 6, (K, B_, H_, W_), generator=g, device=device).float(),
            actions=torch.softmax(torch.randn((K, B_, 9), generator=g, device=device), -1),
            rewards=torch.randn((B_, K), generator=g, dtype=torch.float64, device=device) * 10,
            dones=(torch.rand((B_, K), generator=g, device=device) < 0.2).to(torch.uint8),
            u_next=torch.rand((K, B_, 9), generator=g, device=device),
            u_cur=torch.rand((K, B_, 9), generator=g, device=device)))
    return out


def _half(b, rank, world):
    n = b["rewards"].shape[0] // world
    sl = slice(rank * n, (rank + 1) * n)
    return dict(states=b["states"][:, sl], next_states=b["next_states"][:, sl], actions=b["actions"][:, sl],
                rewards=b["rewards"][sl], dones=b["dones"][sl], u_next=b["u_next"][:, sl], u_cur=b["u_cur"][:, sl])


def _learner(device, seed, **kw):
    from marlnav.maddpg import MADDPG
    hidden = kw.pop("hidden", (16, 16))
    return MADDPG(K, kw.pop("H", H), kw.pop("W", W), hidden=hidden, lr_actor=LR, lr_critic=LR, gamma=0.98, tau=0.1,
                  batch_size=B, device=device, seed=seed, **kw)


def _flat(m):
    return torch.cat([p.detach().reshape(-1).float().cpu() for p in m.state_dict().values()])


def _run(rank, world, outdir, device):
    if device == "cuda":
        torch.cuda.set_device(0)
    shape = dict(H=32, W=32, hidden=(128, 128)) if device == "cuda" else {}
    m = _learner(device, seed=3 + 5 * rank, **shape)  # rank 1's own init is overwritten by the broadcast
    for it, b in enumerate(_batches(device, H_=shape.get("H", H), W_=shape.get("W", W))):
        m.learn(**_half(b, rank, world))
        np.save(os.path.join(outdir, f"w{rank}_{it}.npy"), _flat(m).numpy())


def _worker(rank, world, port, outdir, device):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(rank, world, outdir, device)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(device, d):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, d, device)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes


def _check(device):
    with tempfile.TemporaryDirectory() as d:
        _spawn(device, d)
        two = [[np.load(os.path.join(d, f"w{r}_{it}.npy")) for it in range(UPDATES)] for r in range(2)]
    shape = dict(H=32, W=32, hidden=(128, 128)) if device == "cuda" else {}
    one = _learner(device, seed=3, **shape)
    for it, b in enumerate(_batches(device, H_=shape.get("H", H), W_=shape.get("W", W))):
        one.learn(**b)
        want = _flat(one).numpy()
        np.testing.assert_array_equal(two[0][it], two[1][it])          # identical replicas, every update
        rel = np.linalg.norm(two[0][it] - want) / np.linalg.norm(want)
        assert rel < 1e-4, (it, rel)
        assert np.abs(two[0][it] - want).max() <= 2 * LR * (it + 1)


def test_dp_learner_two_ranks_equal_one_process_cpu():
    _check("cpu")


@pytest.mark.gpu
def test_gpu_dp_learner_two_ranks_equal_one_process():
    _check("cuda")


def _graph_worker(rank, world, port, outdir):
    """Two ranks on one GPU: learners captured as three graph segments with the all-reduces
    between them (fixed half-batches) stay identical to each other and equal the eager DP
    learn on the same inputs (graph replay vs eager: test_gpu_rollout.py's tolerance)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        shape = dict(H=32, W=32, hidden=(128, 128))
        b = _half(_batches("cuda", B_=128, H_=32, W_=32)[0], rank, world)
        batch = (b["states"], b["actions"], b["rewards"], b["next_states"], b["dones"], b["u_next"], b["u_cur"])
        ga = _learner("cuda", seed=1 + rank, capturable=True, **shape)
        ea = _learner("cuda", seed=1 + rank, capturable=True, **shape)
        ga.capture(batch=batch, warmup=2)
        assert ga._graphs is not None  # the segmented form
        for _ in range(2):
            ea.learn(*batch)
        for _ in range(3):
            ga.replay_learn()
            ea.learn(*batch)
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, f"g{rank}.npy"), _flat(ga).numpy())
        np.save(os.path.join(outdir, f"e{rank}.npy"), _flat(ea).numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_dp_graph_segments_equal_eager():
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_graph_worker, args=(r, 2, port, d)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
        assert codes == [0, 0], codes
        g = [np.load(os.path.join(d, f"g{r}.npy")) for r in range(2)]
        e = [np.load(os.path.join(d, f"e{r}.npy")) for r in range(2)]
    np.testing.assert_array_equal(g[0], g[1])
    np.testing.assert_array_equal(e[0], e[1])
    np.testing.assert_allclose(g[0], e[0], rtol=1e-5, atol=1e-6)


def _schedule_worker(rank, world, port, local_envs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from marlnav.train import dp_env_counts, learn_schedule
        g, m = dp_env_counts(local_envs[rank])
        S = -(-200 // g) + 1
        sched = [learn_schedule(i, i + 1, S, g, m, learn_step=10, batch_size=16) for i in range(40)]
        q.put((rank, g, m, sched))
    finally:
        dist.destroy_process_group()


def test_learn_schedule_identical_on_uneven_shards_cpu():
    """with --envs % world != 0 the shards differ by one env; the learn schedule (and
    with it the number of learn() calls, each two gradient all-reduces) must still be the same on
    every rank, or the collectives go out of step.  gloo, world size 2, shards 5 and 4 envs."""
    from marlnav.parallel import shard
    world, G = 2, 9
    local = [shard(G, r, world)[1] for r in range(world)]
    assert local == [5, 4]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_schedule_worker, args=(r, world, port, local, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (_, g0, m0, s0), (_, g1, m1, s1) = res
    assert (g0, m0) == (g1, m1) == (9, 4)
    assert s0 == s1
    # the rule over 9 global envs: learn_step 10 > 9 -> one learn every 10 // 9 = 1 step, once the
    # smallest shard's ring holds a batch of 16 (4 envs x 4 steps)
    assert s0[:3] == [0, 0, 0] and s0[3] == 1


def test_trainer_checkpoint_api():
    """MADDPGAgent's checkpoint API (maddpg/agent.py:255-281) is all there on the trainer."""
    from marlnav.train import MADDPGTrainer
    for name in ("save_checkpoint", "load_checkpoint", "load_wo_memory"):
        assert callable(getattr(MADDPGTrainer, name, None)), name
