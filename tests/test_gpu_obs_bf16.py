"""Lossless compact obs (gw_set_obs_dtype GW_OBS_BF16): every observation value the env writes
(-1, 0, 0.5, 1, 5..13, 9.5) is exact in bfloat16, so the bf16 buffers must equal the float32
path's bit for bit after widening, at reset, every step, for terminal obs, with partial resets,
synchronous and pipelined.  The float32 path itself is pinned to the oracle (test_gpu_parity)."""
import pytest
import torch

from marlnav import _lib
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def _same(x, y):  # y bf16 -> float32; final_obs starts as NaN in both
    y = y.float()
    return int((~((x == y) | (x.isnan() & y.isnan()))).sum())


@pytest.mark.parametrize("name,fear,mode,E", [("grid32", True, False, 4096), ("grid32", True, True, 4096),
                                              ("grid32", False, "lazy", 1000), ("grid64_n8", True, False, 512),
                                              ("level3", True, True, 77)])
def test_bf16_obs_equals_f32(name, fear, mode, E):
    sc = S.builtin(name)
    mk = lambda dt: VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=-5.0, seed=21, final_obs=True,
                               max_steps=30, obs_dtype=dt)
    a, b = mk(torch.float32), mk(torch.bfloat16)
    assert b.out["obs"].dtype == torch.bfloat16
    b.set_obs_async(mode)
    oa, _ = a.reset()
    ob, _ = b.reset()
    b.obs_fence()
    bad = _same(oa, ob)
    for t in range(40):
        r1, r2 = a.step(), b.step()
        b.obs_fence()
        bad += _same(r1.obs, r2.obs) + _same(r1.final_obs, r2.final_obs)
        bad += int((r1.reward != r2.reward).sum())
        if t == 17:
            m = (torch.arange(E, device="cuda") % 4 == 1).to(torch.uint8)
            oa, _ = a.reset(env_mask=m)
            ob, _ = b.reset(env_mask=m)
            bad += _same(oa, ob)
    assert bad == 0
    a.close()
    b.close()


def test_bf16_obs_rejected_without_hw_multiple_of_8():
    # level3 is 10 x 16 = 160 cells (a multiple of 8): a 10 x 15 map is not
    sc = S.compile_scenario(S.level3_like(10, 15, 4, 2))
    with pytest.raises(_lib.GwError):
        VecGridEnv(sc, num_envs=64, obs_dtype=torch.bfloat16)


def test_bf16_rollout_matches_f32():
    """A fused-actor rollout on a bf16-obs env == on the float32 env: same actions / rewards, and
    the (half-size) replay ring holds the same observations."""
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    sc = S.builtin("grid32")
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=5)
    envs = [VecGridEnv(sc, num_envs=2048, fear=True, fear_weight=-5.0, seed=4, final_obs=True, stats=True,
                       obs_dtype=dt) for dt in (torch.float32, torch.bfloat16)]
    ros = [Rollout(e, actors, replay_slots=12, training=True, seed=2, obs_async="lazy") for e in envs]
    for ro in ros:
        ro.reset()
    for _ in range(20):
        r0, r1 = ros[0].step(), ros[1].step()
    for ro in ros:
        ro.fence()
    assert torch.equal(ros[0].replay.obs, ros[1].replay.obs.float())
    assert torch.equal(ros[0].replay.final_obs, ros[1].replay.final_obs.float())
    assert torch.equal(ros[0].replay.reward, ros[1].replay.reward)
    assert torch.equal(ros[0].replay.probs, ros[1].replay.probs)
    s0 = ros[0].replay.sample(64, generator=torch.Generator(device="cuda").manual_seed(1))
    s1 = ros[1].replay.sample(64, generator=torch.Generator(device="cuda").manual_seed(1))
    assert s1[0].dtype == torch.float32 and all(torch.equal(x, y) for x, y in zip(s0, s1))
    assert ros[0].totals() == ros[1].totals()
    for e in envs:
        e.close()


@pytest.mark.parametrize("path", ["merged", "defer"])
def test_bf16_pipelined_ring_equals_f32(path, monkeypatch):
    """bf16 obs through the step pipeline with no fence inside the loop (every step's obs into
    its own ring slot; with GW_KERNEL=merged each step is one step_obs launch whose writer role
    produces the previous step's bf16 obs) == the synchronous float32 env."""
    monkeypatch.setenv("GW_KERNEL", path)
    sc = S.builtin("grid32")
    E, T = 3000, 24
    a = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=31, final_obs=True, max_steps=20)
    b = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=31, final_obs=True, max_steps=20,
                   obs_dtype=torch.bfloat16)
    b.set_obs_async(True)
    ring = torch.empty((T, sc.K, E, sc.H, sc.W), dtype=torch.bfloat16, device="cuda")
    fin = torch.full((T, sc.K, E, sc.H, sc.W), -3.0, dtype=torch.bfloat16, device="cuda")
    ref = torch.empty((T, sc.K, E, sc.H, sc.W), dtype=torch.float32, device="cuda")
    reff = torch.full((T, sc.K, E, sc.H, sc.W), -3.0, dtype=torch.float32, device="cuda")
    a.reset()
    b.reset()
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(T):
        r1 = a.step(obs_out=ref[t], final_obs_out=reff[t])
        r2 = b.step(obs_out=ring[t], final_obs_out=fin[t])
        bad += (r1.reward != r2.reward).sum() + (r1.done != r2.done).sum() + (r1.shaped != r2.shaped).sum()
    b.obs_fence()
    bad += (ref != ring.float()).sum() + (reff != fin.float()).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    a.close()
    b.close()
