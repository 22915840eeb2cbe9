"""The multi-rank rollout path on the GPU: 2 ranks on one MI355X.

RCCL refuses two ranks on one device, so the ranks use the gloo backend on CUDA tensors (the
same torch.distributed calls bench.py / Rollout issue under RCCL on an 8-GPU node).  What runs
on the GPU is the product path: each rank steps its contiguous shard of global env ids with
the HIP env, the step kernels' running statistics total (gw_step_out.stats_acc, all-reduced
once when Rollout.totals() reads it: no per-step reduction launch) and the ReturnGather
(ep_return / done written by gw_step straight into the send buffer, one all_gather_into_tensor
per step, device-side compaction).  The sharded run must
equal ONE process stepping all envs: identical completed-episode returns in the reference's
order (maddpg/agent.py:229-247: step, then env id) on every rank, identical positions, and the
same statistics (sums in a different order: rtol 1e-12).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

G, STEPS, SEED = 4099, 60, 9   # ragged shards (2050 + 2049)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, outdir, fused_actor):
    from marlnav.parallel import ReturnGather, shard
    from marlnav.rollout import Rollout
    from marlnav.vec_env import VecGridEnv
    torch.cuda.set_device(0)
    off, cnt = shard(G, rank, world)
    env = VecGridEnv("grid32", num_envs=cnt, fear=True, fear_weight=-5.0, max_steps=40, seed=SEED,
                     env_offset=off, stats=True)
    actors = None
    if fused_actor:  # the C5 rollout: fused actor, replay ring, lazy async obs
        from marlnav.actor import MultiAgentActors
        actors = MultiAgentActors(env.K, env.H, env.W, "mlp", device="cuda", seed=0)
    gat = ReturnGather(G, rank, world, "cuda", window=16)
    ro = Rollout(env, actors, replay_slots=8 if fused_actor else 0, seed=0, obs_async="lazy" if fused_actor else True,
                 gather=gat)
    ro.reset()
    for _ in range(STEPS):
        ro.step()
    ro.fence()
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, f"scores{rank}.npy"), ro.completed_scores())
    np.save(os.path.join(outdir, f"totals{rank}.npy"), np.array(list(ro.totals().values())))
    np.save(os.path.join(outdir, f"pos{rank}.npy"), env.positions().cpu().numpy())
    env.close()


def _worker(rank, world, port, outdir, fused_actor):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(rank, world, outdir, fused_actor)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fused_actor", [False, True])
def test_two_ranks_equal_one_process(fused_actor):
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, d, fused_actor)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
        assert codes == [0, 0], codes
        os.makedirs(os.path.join(d, "one"))
        _run(0, 1, os.path.join(d, "one"), fused_actor)
        one = {n: np.load(os.path.join(d, "one", f"{n}0.npy")) for n in ("scores", "totals", "pos")}
        two = [{n: np.load(os.path.join(d, f"{n}{r}.npy")) for n in ("scores", "totals", "pos")} for r in range(2)]
    assert len(one["scores"]) > 100
    for r in range(2):
        np.testing.assert_array_equal(two[r]["scores"], one["scores"])        # gathered == single run
        np.testing.assert_allclose(two[r]["totals"], one["totals"], rtol=1e-12)  # all-reduced stats
    pos = np.concatenate([two[0]["pos"], two[1]["pos"]], axis=0)  # [E, N] shards
    np.testing.assert_array_equal(pos, one["pos"])
    # the gathered list is the per-step list of the totals' completed episodes
    assert len(one["scores"]) == int(one["totals"][1])
    np.testing.assert_allclose(one["scores"].sum(), one["totals"][0], rtol=1e-12)
