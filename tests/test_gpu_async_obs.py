"""Async obs writes (gw_set_obs_async: the obs writer of step t overlaps the world update of
step t+1, descriptors double-buffered) == the synchronous path, bit for bit.

No host synchronisation inside the stepping loops: every step's obs goes to its own slot and
every other output is cloned on the caller's stream right after the step, so a missing
dependency (descriptor WAR, join, fence) shows up as a mismatch instead of being hidden by
an idle GPU.  The synchronous path itself is pinned to the oracle in test_gpu_parity.py.
"""
import pytest
import torch

from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu

OUTS = ("reward", "fear", "shaped", "term", "trunc", "done", "mask", "ep_return", "actions", "final_pos")


@pytest.mark.parametrize("path,fear,name,mode,E", [
    ("defer", True, "grid32", True, 4096), ("defer", False, "grid32", True, 4096),
    ("defer", True, "grid64_n8", True, 1024), ("defer", True, "grid32", "lazy", 4096),
    ("defer", False, "grid32", "lazy", 4096), ("defer", False, "grid64_n8", True, 1024),
    ("defer", True, "level3", True, 1), ("defer", True, "level3", "lazy", 333),   # ragged env counts
    ("defer", True, "grid32", True, 515), ("defer", False, "grid32", True, 257),
    # merged: one step_obs launch per step (step t + the obs writer of step t-1), one stream
    ("merged", True, "grid32", True, 4096), ("merged", False, "grid32", True, 4099),
    ("merged", True, "grid64_n8", "lazy", 1024), ("merged", True, "level3", True, 1),
    ("merged", False, "level3", True, 333)])
def test_async_obs_matches_sync(path, fear, name, mode, E, monkeypatch):
    monkeypatch.setenv("GW_KERNEL", path)
    sc = S.builtin(name)
    T = 12 if name == "grid64_n8" else 24
    mk = lambda: VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=5, final_obs=True, debug=True,
                            stats=True)
    a, b = mk(), mk()
    b.set_obs_async(mode)
    shape = (T, sc.K, E, sc.H, sc.W)
    obs_a = torch.empty(shape, dtype=torch.float32, device="cuda")
    fin_a = torch.full(shape, -7.0, dtype=torch.float32, device="cuda")
    obs_b = torch.empty(shape, dtype=torch.float32, device="cuda")
    fin_b = torch.full(shape, -7.0, dtype=torch.float32, device="cuda")
    ra, rb = a.reset(), b.reset()
    b.obs_fence()
    assert torch.equal(ra[0], rb[0])
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(T):
        r1 = a.step(obs_out=obs_a[t], final_obs_out=fin_a[t])
        r2 = b.step(obs_out=obs_b[t], final_obs_out=fin_b[t])
        for n in OUTS:  # stream-ordered without any fence
            bad += (getattr(r1, n) != getattr(r2, n)).sum()
        bad += (r1.stats.sum(0) != r2.stats.sum(0)).sum()
        if t == T // 2:  # a partial reset in the middle of the pipeline fences itself
            m = (torch.arange(E, device="cuda") % 3 == 0).to(torch.uint8)
            a.reset(env_mask=m)
            b.reset(env_mask=m)
    b.obs_fence()
    bad += (obs_a != obs_b).sum() + (fin_a != fin_b).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    # a step without obs outputs in the middle of the pipeline (the in-place descriptor path)
    a.set_obs_async(True)
    a.step(obs_out=obs_a[0])
    b.step(obs_out=obs_b[0])
    for env in (a, b):  # gw_step with no outputs at all (null gw_step_out)
        assert env.lib.gw_step(env.handle, None, None, None, None, env._stream()) == 0
    r1 = a.step(obs_out=obs_a[1])
    r2 = b.step(obs_out=obs_b[1])
    a.obs_fence()
    b.obs_fence()
    bad += (obs_a[:2] != obs_b[:2]).sum() + (r1.reward != r2.reward).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    a.set_obs_async(False)
    # the same state afterwards; switching async off drains the writer
    sa, sb = a.state(), b.state()
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    b.set_obs_async(False)
    r1, r2 = a.step(), b.step()
    torch.cuda.synchronize()
    assert torch.equal(r1.obs, r2.obs) and torch.equal(r1.reward, r2.reward)
    a.close()
    b.close()


@pytest.mark.parametrize("mode,fear_async,path", [(True, False, "defer"), ("lazy", False, "defer"),
                                                  ("lazy", True, "defer"), (True, True, "defer"),
                                                  ("lazy", False, "merged"), (True, True, "merged")])
def test_async_rollout_fused_actor_matches_sync(mode, fear_async, path, monkeypatch):
    """Rollout(obs_async) with the fused actor (reads the alternating descriptors) == the
    synchronous rollout: same actions, probs, rewards and replay-ring contents."""
    monkeypatch.setenv("GW_KERNEL", path)
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    E = 4096
    torch.manual_seed(0)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=9)
    envs = [VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=3, final_obs=True, stats=True)
            for _ in range(2)]
    ros = [Rollout(envs[0], actors, replay_slots=40, training=True, seed=4, obs_async=False),
           Rollout(envs[1], actors, replay_slots=40, training=True, seed=4, obs_async=mode,
                   fear_async=fear_async)]
    assert all(ro.fused for ro in ros)
    for ro in ros:
        ro.reset()
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(30):
        r0, r1 = ros[0].step(), ros[1].step()
        bad += (r0.done != r1.done).sum() + (r0.mask != r1.mask).sum()
        if not fear_async:  # else the FeAR outputs are ordered by the next step / fence
            bad += (r0.shaped != r1.shaped).sum()
    for ro in ros:
        ro.fence()
    for name in ("obs", "final_obs", "probs", "reward", "term", "done", "t_dev"):
        bad += (getattr(ros[0].replay, name) != getattr(ros[1].replay, name)).sum()
    st0, st1 = envs[0].state(), envs[1].state()
    bad += sum((st0[k] != st1[k]).sum() for k in st0)
    torch.cuda.synchronize()
    assert int(bad) == 0
    t0, t1 = ros[0].totals(), ros[1].totals()
    assert t0 == t1
    for e in envs:
        e.close()


def test_fear_async_env_outputs_after_fence():
    """gw_set_obs_async(| 4): the FeAR-owned outputs of every step equal the synchronous env's
    once fenced, with no host synchronisation in the loop (the fence is stream-ordered)."""
    sc = S.builtin("grid32")
    E, T = 4096, 20
    mk = lambda: VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=8, stats=True)
    a, b = mk(), mk()
    b.set_obs_async("lazy", fear_async=True)
    a.reset()
    b.reset()
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(T):
        r1, r2 = a.step(), b.step()
        bad += (r1.done != r2.done).sum() + (r1.reward != r2.reward).sum()
        b.fear_fence()
        for n in ("fear", "shaped", "ep_return", "ep_fear"):
            bad += (getattr(r1, n) != getattr(r2, n)).sum()
        bad += (r1.stats.sum(0) != r2.stats.sum(0)).sum()
    b.obs_fence()
    bad += (a.out["obs"] != b.out["obs"]).sum()
    sa, sb = a.state(), b.state()
    bad += sum((sa[k] != sb[k]).sum() for k in sa)
    torch.cuda.synchronize()
    assert int(bad) == 0
    a.close()
    b.close()


@pytest.mark.parametrize("mode", [True, "lazy"])
def test_async_obs_same_buffer_every_step(mode):
    """Async writers of consecutive steps into the SAME buffers (the env's own obs / final_obs,
    two obs streams): the write-after-write order holds, the buffers end as the last step's."""
    sc = S.builtin("grid32")
    E, T = 4096, 15
    mk = lambda: VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=12, final_obs=True, stats=True)
    a, b = mk(), mk()
    b.set_obs_async(mode)
    a.reset()
    b.reset()
    for t in range(T):
        r1, r2 = a.step(), b.step()
    b.obs_fence()
    differ = lambda x, y: (~((x == y) | (x.isnan() & y.isnan()))).sum()  # final_obs starts as NaN
    bad = differ(r1.obs, r2.obs) + differ(r1.final_obs, r2.final_obs) + (r1.reward != r2.reward).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    a.close()
    b.close()


def test_async_obs_alternating_buffers():
    """Double-buffered obs outputs (step t into buffer t & 1, e.g. replay slots): every buffer
    holds the obs of the last step that wrote it."""
    sc = S.builtin("grid32")
    E, T = 4096, 16
    a = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=13)
    b = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=13)
    b.set_obs_async(True)
    bufs = [b.out["obs"], torch.empty_like(b.out["obs"])]
    a.reset()
    b.reset()
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    last = [None, None]
    for t in range(T):
        r1 = a.step()
        b.step(obs_out=bufs[t & 1])
        last[t & 1] = r1.obs.clone()
    b.obs_fence()
    for i in range(2):
        bad += (last[i] != bufs[i]).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    a.close()
    b.close()


@pytest.mark.parametrize("ring,same_final", [(3, False), (2, True), (5, True)])
def test_async_obs_rings_and_shared_final_buffer(ring, same_final, monkeypatch):
    """The writers of consecutive steps go to alternating obs streams only when both their obs and
    final_obs buffers differ; a ring of 3 / 5 slots reuses a slot on the OTHER stream two steps
    later (ordered through the descriptor WAR chain), and a final_obs buffer shared by every step
    keeps the writers on one stream.  Every slot holds the obs of the last step that wrote it."""
    monkeypatch.setenv("GW_KERNEL", "defer")
    sc = S.builtin("grid32")
    E, T = 4096, 17
    a = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=23, max_steps=10, final_obs=True)
    b = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=23, max_steps=10, final_obs=True)
    b.set_obs_async(True)
    obs = [torch.empty_like(b.out["obs"]) for _ in range(ring)]
    fin = [torch.full_like(b.out["obs"], -3.0) for _ in range(1 if same_final else ring)]
    ref_fin = [torch.full_like(a.out["obs"], -3.0) for _ in range(len(fin))]
    a.reset()
    b.reset()
    last = [None] * ring
    for t in range(T):
        ra = a.step(final_obs_out=ref_fin[t % len(ref_fin)])
        b.step(obs_out=obs[t % ring], final_obs_out=fin[t % len(fin)])
        last[t % ring] = ra.obs.clone()
    b.obs_fence()
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    for i in range(ring):
        bad += (last[i] != obs[i]).sum()
    for x, y in zip(ref_fin, fin):
        bad += (x != y).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    a.close()
    b.close()


@pytest.mark.parametrize("chunks,mode,E", [(2, True, 4099), (4, True, 4096), (3, "lazy", 1000)])
def test_async_obs_chunked_writer(chunks, mode, E, monkeypatch):
    """GW_OBS_CHUNKS: each step's writer as several launches over consecutive env ranges (the
    C5 / c4cnn default, so the next actor's kernels are dispatched between them) == sync."""
    monkeypatch.setenv("GW_OBS_CHUNKS", str(chunks))
    test_async_obs_matches_sync("defer", True, "grid32", mode, E, monkeypatch)


@pytest.mark.parametrize("chunks", [2, 4])
def test_async_rollout_chunked_writer_matches_sync(chunks, monkeypatch):
    """The C5 default pipeline (eager writer in GW_OBS_CHUNKS launches, replay-ring slots on
    alternating obs streams, fused actor) == the synchronous rollout."""
    monkeypatch.setenv("GW_OBS_CHUNKS", str(chunks))
    test_async_rollout_fused_actor_matches_sync(True, False, "defer", monkeypatch)
