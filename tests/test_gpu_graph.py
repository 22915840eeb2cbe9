"""Graph-replayed steps (VecGridEnv.capture_steps) == eager steps, bit for bit.

C2-sized workloads are bound by the host's launch chain, so bench.py replays their timed steps
as HIP graphs of n captured gw_step calls (synchronous obs; the per-step return gather and its
window compaction inside the graph).  Two envs with the same seed: one stepped eagerly, one by
graph replays; after every replay every output of the last step, the env state and the
gathered completed-episode returns must be identical.  FeAR on exercises the synchronous
defer path's fork / join through the aux stream inside the capture."""
import numpy as np
import pytest
import torch

from marlnav.parallel import ReturnGather
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu

OUTS = ("obs", "reward", "fear", "shaped", "term", "trunc", "done", "mask", "crashes", "apples", "ep_return",
        "ep_fear", "ep_len", "stats")


@pytest.mark.parametrize("scenario,E,fear,n,path,async_obs", [
    ("grid32", 1000, False, 8, "defer", False), ("grid32", 777, True, 6, "defer", False),
    ("grid64_n8", 300, True, 4, "defer", False), ("level3", 1, False, 16, "defer", False),
    # merged async: each captured step is one step_obs launch (step t + the writer of step t-1)
    ("grid32", 4096, False, 8, "merged", True), ("grid32", 999, True, 6, "merged", True),
    ("grid64_n8", 200, True, 4, "merged", True)])
def test_graph_replay_equals_eager(scenario, E, fear, n, path, async_obs, monkeypatch):
    monkeypatch.setenv("GW_KERNEL", path)
    envs, gathers = [], []
    for i in range(2):
        env = VecGridEnv(scenario, num_envs=E, fear=fear, fear_weight=-5.0, max_steps=12, seed=5, stats=True)
        if async_obs and i == 1:
            env.set_obs_async(True)
        env.reset()
        envs.append(env)
        gathers.append(ReturnGather(E, 0, 1, env.device, window=n))
    eager, graphed = envs
    for i in range(3):  # a few eager steps first on both: the capture starts mid-episode
        for env, g in zip(envs, gathers):
            env.step(into=g.into())
            g.push()
    for g in gathers:
        g.compact()
    graph = graphed.capture_steps(n, gathers[1])
    episodes = 0
    for rep in range(4):
        for _ in range(n):
            eager.step(into=gathers[0].into())
            gathers[0].push()
        graph.replay()
        graphed.obs_fence()  # async: the last captured step's writer
        torch.cuda.synchronize()
        for name in OUTS:
            a, b = eager.out[name], graphed.out[name]
            assert torch.equal(a, b), (rep, name)
        # the gather's last slot is where the step wrote its returns / dones
        sa, sb = eager.state(), graphed.state()
        for k in sa:
            assert torch.equal(sa[k], sb[k]), (rep, k)
        ca, cb = gathers[0].completed(), gathers[1].completed()
        np.testing.assert_array_equal(ca, cb)
        episodes = len(ca)
    assert episodes > 0 or E == 1
    for env in envs:
        env.close()


def test_capture_rejects_async_obs_off_the_merged_path(monkeypatch):
    monkeypatch.setenv("GW_KERNEL", "defer")
    env = VecGridEnv("grid32", num_envs=64, fear=False, seed=1)
    env.set_obs_async(True)
    env.reset()
    with pytest.raises(Exception, match="synchronous obs"):
        env.capture_steps(4)
    env.close()


def test_merged_capture_needs_even_steps_after_a_step(monkeypatch):
    monkeypatch.setenv("GW_KERNEL", "merged")
    env = VecGridEnv("grid32", num_envs=64, fear=False, seed=1)
    env.set_obs_async(True)
    env.reset()
    with pytest.raises(Exception, match="even n"):
        env.capture_steps(4)  # no step since the reset: no writer queued
    env.step()
    with pytest.raises(Exception, match="even n"):
        env.capture_steps(3)
    env.close()
