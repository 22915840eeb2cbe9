"""C2 as BASELINE names it (``bench.py --config c2``): the MADDPG rollout with the configs/mlp.yaml
actors acting on the full-grid obs every step (maddpg/agent.py:89, 109-127, 190-197) at 4,096 envs,
FeAR off (configs/custom.yaml, weight -2), replayed as HIP graphs (``Rollout.capture``: one graph
of 16 steps per phase of the replay ring, the fused actor's noise counter read from the ring's
device step count).

1. The graph-replayed rollout == the eager rollout bit for bit: the whole replay ring (obs,
   terminal obs, action probabilities, shaped rewards, terminations, dones), the env state, the
   statistics totals and the gathered completed-episode list, after 5 eager warmup steps, every
   ring-phase graph replayed (graph 0 twice: the cycle closes) and eager steps after them.
2. The eager rollout == the C oracle fed the actions the actor chose (``vec_step(rl_act=...)``):
   every step's shaped rewards (the ring's reward slots), terminations and dones for all 4,096
   envs, and the observations of every ring slot written in the last SLOTS steps.
"""
import numpy as np
import pytest
import torch

from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv
from oracle import oracle as O

pytestmark = pytest.mark.gpu

E, CAP, SEED, G, WARM = 4096, 150, 42, 16, 5
SLOTS = 64                       # -(-200_000 // 4096) + 1 = 50, rounded up to a multiple of G
T = WARM + (SLOTS // G + 1) * G + 3


def _rollout(graph: bool):
    from marlnav.maddpg import MADDPG
    from marlnav.parallel import ReturnGather
    from marlnav.rollout import Rollout
    mp = pytest.MonkeyPatch()
    mp.delenv("GW_KERNEL", raising=False)
    mp.setenv("GW_OBS_CHUNKS", "2")  # bench.py's rollout default (read by gw_create)
    try:
        env = VecGridEnv("grid32", num_envs=E, fear=False, fear_weight=-2.0, max_steps=CAP, auto_reset=True,
                         seed=SEED, stats=True)
    finally:
        mp.undo()
    assert env.kernel_path == "merged"
    learner = MADDPG(env.K, env.H, env.W, device=env.device, seed=0, capturable=True)
    gather = ReturnGather(E, 0, 1, env.device, window=G)
    ro = Rollout(env, learner.actors, replay_slots=SLOTS, training=True, seed=SEED, obs_async=True, gather=gather)
    assert ro.fused
    ro.reset()
    acts = []
    t = 0
    while t < T:
        if graph and t == WARM:
            gather.compact()
            graphs = ro.capture(G)
            assert len(graphs.graphs) == SLOTS // G
        if graph and WARM <= t and t + G <= T - 3:
            graphs.replay()
            t += G
            continue
        ro.step()
        acts.append((t, ro._actions.clone()))
        t += 1
    ro.fence()
    rp = ro.replay
    out = {n: getattr(rp, n).clone() for n in ("obs", "final_obs", "probs", "reward", "term", "done")}
    out["state"] = env.state()
    out["totals"] = ro.totals()
    out["scores"] = ro.completed_scores()
    out["t"] = (ro.t, rp.t, int(rp.t_dev), ro._calls)
    torch.cuda.synchronize()
    env.close()
    return out, acts


@pytest.fixture(scope="module")
def runs():
    return _rollout(False), _rollout(True)


def test_graph_rollout_equals_eager(runs):
    (a, _), (b, _) = runs
    assert a["t"] == b["t"] == (T, T, T, T)
    for n in ("obs", "final_obs", "probs", "reward", "term", "done"):
        assert torch.equal(a[n], b[n]), n
    for n, v in a["state"].items():
        assert torch.equal(v, b["state"][n]), n
    assert a["totals"] == b["totals"]
    np.testing.assert_array_equal(a["scores"], b["scores"])
    assert len(a["scores"]) > 1000


def test_eager_rollout_matches_oracle(runs):
    (a, acts), _ = runs
    assert len(acts) == T
    sc = S.builtin("grid32")
    orc = O.OracleEnvs(sc, E, fear=False, fear_weight=-2.0, max_steps=CAP, seed=SEED, reset=False)
    obs = np.zeros((sc.K, E, sc.HW), np.float32)
    orc.reset_all(obs=obs, nthreads=16)
    outs = (O.StepOut * E)()
    K = sc.K
    ring_obs = a["obs"].cpu().numpy().reshape(SLOTS, K, E, -1)
    reward = a["reward"].cpu().numpy()
    term = a["term"].cpu().numpy()
    done = a["done"].cpu().numpy()
    fin = a["final_obs"].cpu().numpy().reshape(SLOTS, K, E, -1)
    for t, act in acts:
        fobs = np.zeros_like(obs)
        orc.vec_step(act.cpu().numpy(), obs=obs, final_obs=fobs, outs=outs, nthreads=16)
        slot = t % SLOTS
        if t >= T - SLOTS:  # obs_{t+1} in slot t + 1 (written by the next step_obs or the fence)
            np.testing.assert_array_equal(ring_obs[(t + 1) % SLOTS], obs, err_msg=f"ring obs after step {t}")
            dn = np.array([outs[e].done for e in range(E)], bool)
            np.testing.assert_array_equal(fin[slot][:, dn], fobs[:, dn], err_msg=f"terminal obs of step {t}")
        if t >= T - SLOTS + 1:  # the ring slots not overwritten since
            o = [outs[e] for e in range(E)]
            np.testing.assert_array_equal(reward[slot], np.array([list(x.shaped)[:K] for x in o]),
                                          err_msg=f"shaped reward at step {t}")
            np.testing.assert_array_equal(term[slot], np.array([list(x.term)[:K] for x in o], np.uint8),
                                          err_msg=f"term at step {t}")
            np.testing.assert_array_equal(done[slot], np.array([x.done for x in o], np.uint8),
                                          err_msg=f"done at step {t}")
    np.testing.assert_array_equal(ring_obs[T % SLOTS], obs, err_msg="the last step's obs in the ring")


@pytest.mark.parametrize("arch,scen,P,fear", [("cnn", "grid64_n8", 16, False), ("mlp", "grid32", 11, True)])
def test_window_rollout_graph_equals_eager(arch, scen, P, fear):
    """The local-window rollouts (bench c4patch: the configs/cnn.yaml head on 16 x 16 windows of the
    64 x 64 / N = 8 grid, window writer on a side stream; c5patch: the MLP actors on 11 x 11
    windows, FeAR on) replayed as ring-phase graphs == the same rollout stepped eagerly, bit for
    bit (ring contents, env state, totals)."""
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    En, slots, warm = 1024, 32, 3
    steps = warm + (slots // G + 1) * G + 2
    outs = []
    for graph in (False, True):
        env = VecGridEnv(scen, num_envs=En, fear=fear, fear_weight=-5.0, max_steps=40, auto_reset=True, seed=SEED,
                         stats=True, obs=False)
        actors = MultiAgentActors(env.K, P, P, arch=arch, device=env.device, seed=0)
        ro = Rollout(env, actors, replay_slots=slots, training=True, seed=SEED, patch=P)
        assert ro.fused
        ro.reset()
        t = 0
        while t < steps:
            if graph and t == warm:
                graphs = ro.capture(G)
            if graph and warm <= t and t + G <= steps - 2:
                graphs.replay()
                t += G
                continue
            ro.step()
            t += 1
        ro.fence()
        rp = ro.replay
        o = {n: getattr(rp, n).clone() for n in ("obs", "final_obs", "probs", "reward", "term", "done")}
        o["state"] = env.state()
        o["totals"] = ro.totals()
        torch.cuda.synchronize()
        env.close()
        outs.append(o)
    a, b = outs
    for n in ("obs", "final_obs", "probs", "reward", "term", "done"):
        assert torch.equal(a[n], b[n]), n
    for n, v in a["state"].items():
        assert torch.equal(v, b["state"][n]), n
    assert a["totals"] == b["totals"]


@pytest.mark.parametrize("arch,scen,P,fear", [("cnn", "grid64_n8", 16, False)])
def test_window_graph_captured_right_after_reset(arch, scen, P, fear):
    """a capture taken right after reset() (no listing pending) followed by EAGER steps
    before the first replay, then replays, then eager steps again: == the eager rollout bit for bit.
    The CNN head's listing never crosses a graph boundary (Rollout.capture), and the capture leaves
    the host's listing state (_lists_ready, the actor's pending flag) as it found it."""
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    En, slots = 1024, 32
    plan = ["capture"] + ["e"] * G + ["g", "g"] + ["e"] * 3
    outs = []
    for graph in (False, True):
        env = VecGridEnv(scen, num_envs=En, fear=fear, fear_weight=-5.0, max_steps=40, auto_reset=True, seed=SEED,
                         stats=True, obs=False)
        actors = MultiAgentActors(env.K, P, P, arch=arch, device=env.device, seed=0)
        ro = Rollout(env, actors, replay_slots=slots, training=True, seed=SEED, patch=P)
        assert ro.fused and ro._cnn_list
        ro.reset()
        for op in plan:
            if op == "capture":
                if graph:
                    graphs = ro.capture(G)
                    assert ro._lists_ready is False and not actors._fast.get("pending")
            elif op == "g" and graph:
                graphs.replay()
            elif op == "g":
                for _ in range(G):
                    ro.step()
            else:
                ro.step()
        ro.fence()
        rp = ro.replay
        o = {n: getattr(rp, n).clone() for n in ("obs", "final_obs", "probs", "reward", "term", "done")}
        o["state"] = env.state()
        o["totals"] = ro.totals()
        torch.cuda.synchronize()
        env.close()
        outs.append(o)
    a, b = outs
    for n in ("obs", "final_obs", "probs", "reward", "term", "done"):
        assert torch.equal(a[n], b[n]), n
    for n, v in a["state"].items():
        assert torch.equal(v, b["state"][n]), n
    assert a["totals"] == b["totals"]
