"""The C5 and C2 bench modes, exactly as bench.py runs them, pinned to the C oracle.

C5 (``bench.py --config c5``, one rank's workload): the LAST shard of the 8-GPU run, global envs
[7 * 65,536, 8 * 65,536) (``env_offset = 7 * 65536``: every draw is keyed by the global env id), FeAR
on (weight -5), 150-step cap, seed 42; the fused actor (gw_actor_act over the obs descriptors, the
MADDPG actors built from seed 0 as bench.py builds them), obs writes pipelined with the next step
as 2 launches (``GW_OBS_CHUNKS=2``, eager), the zero-copy replay ring of MEMORY_SIZE 200,000
(5 slots of 65,536 envs) and the per-step return gather (``ReturnGather.into()``: the step writes
ep_return / done into the gather's buffers).  The actions the actor chose are recorded and
replayed into the oracle (``vec_step(rl_act=...)``): positions, rewards, FeAR, shaped rewards
(the ring's reward slots), terminations (the ring's term slots), dones (the ring's done slots and
the gather's), ep_return (the gather's), every observation (the ring's obs slots) and terminal
observation (the ring's final-obs slots) of a slice that straddles every kernel's block edges
and of envs whose episode ran into the cap are compared bit for bit.  Over all 65,536 envs the
gathered completed-episode list equals the per-step done envs' returns in the reference's order
(maddpg/agent.py:229-247).

C2's env alone (``bench.py --config c2env``): 4,096 envs, FeAR off (weight -2), the merged ``step_obs`` path with
async obs, 5 eager warmup steps, then the timed steps as replays of a 16-step HIP graph
(``VecGridEnv.capture_steps(16, gather)``) whose gather window is compacted inside the graph.  The
oracle steps all 4,096 envs with the device RNG's policies (native mode): positions after every
replay, every step's ep_return / done (the gather's receive window after each replay), the last
step's outputs, the final observation, and the completed-episode list, bit for bit.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu

E5, OFF5, T5, CAP, SEED = 65536, 7 * 65536, 165, 150, 42
SLICE0, SLICE = 4096 - 128, 256


def _c5_run(sel_capped: np.ndarray | None):
    """One C5-mode rollout of T5 steps; records the selected envs' per-step outputs."""
    from marlnav.maddpg import MADDPG
    from marlnav.parallel import ReturnGather
    from marlnav.rollout import Rollout
    env = VecGridEnv("grid32", num_envs=E5, fear=True, fear_weight=-5.0, max_steps=CAP, auto_reset=True, seed=SEED,
                     env_offset=OFF5, stats=True)
    dev = env.device
    learner = MADDPG(env.K, env.H, env.W, device=dev, seed=0, capturable=True)
    gather = ReturnGather(E5, 0, 1, dev)
    ro = Rollout(env, learner.actors, replay_slots=-(-200_000 // E5) + 1, training=True, seed=SEED,
                 obs_async=True, gather=gather)
    assert ro.fused and env.obs_async and env.kernel_path == "defer"
    S_ = ro.replay.S
    sel = np.arange(SLICE0, SLICE0 + SLICE) if sel_capped is None else \
        np.concatenate([np.arange(SLICE0, SLICE0 + SLICE), sel_capped])
    idx = torch.as_tensor(sel, device=dev)
    rp = ro.replay
    ro.reset()
    ro.fence()
    rec = {n: [] for n in ("act", "pos", "reward", "fear", "shaped", "term", "trunc", "done",
                           "ep_return", "ep_len", "obs", "final_obs")}
    rec["reset_obs"] = rp.obs[0][:, idx].clone()
    all_done, all_ret, all_len = [], [], []
    for t in range(T5):
        r = ro.step()
        cur = t % S_
        rec["act"].append(ro._actions[idx].clone())
        rec["pos"].append(env.state()["pos"][:, idx].clone())
        for n in ("reward", "fear", "trunc", "ep_len"):
            rec[n].append(getattr(r, n)[idx].clone())
        rec["shaped"].append(rp.reward[cur][idx].clone())
        rec["term"].append(rp.term[cur][idx].clone())
        assert r.done.data_ptr() == rp.done[cur].data_ptr()  # the step wrote done into the ring slot
        rec["done"].append(r.done[idx].clone())
        rec["ep_return"].append(r.ep_return[idx].clone())       # the gather's buffer
        all_done.append(r.done.clone())
        all_ret.append(r.ep_return.clone())
        all_len.append(r.ep_len.clone())
        if t % 4 == 3 or t == T5 - 1:  # fence every 4 steps: slots of the last 4 steps still intact (S = 5)
            ro.fence()
            for u in range(t - (t % 4), t + 1):
                rec["obs"].append(rp.obs[(u + 1) % S_][:, idx].clone())
                rec["final_obs"].append(rp.final_obs[u % S_][:, idx].clone())
    ro.fence()
    scores = ro.completed_scores()
    torch.cuda.synchronize()
    host = {n: torch.stack(v).cpu().numpy() for n, v in rec.items() if isinstance(v, list)}
    host["reset_obs"] = rec["reset_obs"].cpu().numpy()
    done = torch.stack(all_done).cpu().numpy()
    ret = torch.stack(all_ret).cpu().numpy()
    ep_len = torch.stack(all_len).cpu().numpy()
    env.close()
    return sel, host, done, ret, ep_len, scores


@pytest.fixture(scope="module")
def c5_run():
    mp = pytest.MonkeyPatch()
    mp.delenv("GW_KERNEL", raising=False)
    mp.setenv("GW_OBS_CHUNKS", "2")  # bench.py's C5 default (read by gw_create)
    try:
        _, _, done, _, ep_len, _ = _c5_run(None)
        capped = np.nonzero(((ep_len == CAP) & (done != 0)).any(0))[0]
        capped = capped[(capped < SLICE0) | (capped >= SLICE0 + SLICE)][:16]
        return _c5_run(capped) + (capped,)
    finally:
        mp.undo()


def _oracle_replay(sc, goff, acts):
    """Oracle outputs of `count` global envs starting at goff, RL actions [T, count, K]."""
    T, count = acts.shape[0], acts.shape[1]
    orc = O.OracleEnvs(sc, count, fear=True, fear_weight=-5.0, max_steps=CAP, seed=SEED, env_offset=goff, reset=False)
    obs = np.zeros((sc.K, count, sc.HW), np.float32)
    orc.reset_all(obs=obs, nthreads=16)
    res = {n: [] for n in ("pos", "reward", "fear", "shaped", "term", "trunc", "done", "ep_return", "ep_len", "obs",
                           "final_obs")}
    res["reset_obs"] = obs.copy()
    outs = (O.StepOut * count)()
    K = sc.K
    for t in range(T):
        fin = np.full((sc.K, count, sc.HW), np.nan, np.float32)
        orc.vec_step(acts[t], obs=obs, outs=outs, nthreads=16, final_obs=fin)
        o = [outs[e] for e in range(count)]
        for n in ("reward", "fear", "shaped", "term", "trunc"):
            res[n].append([list(getattr(x, n))[:K] for x in o])
        res["done"].append([x.done for x in o])
        res["ep_return"].append([x.ep_return for x in o])
        res["ep_len"].append([x.ep_len for x in o])
        res["pos"].append(orc.positions().T.copy())
        res["obs"].append(obs.copy())
        res["final_obs"].append(fin)
    return {n: np.asarray(v) for n, v in res.items()}


def _check_c5(host, cols, ref, what):
    a = host
    for n in ("reward", "fear", "shaped", "term", "trunc"):
        np.testing.assert_array_equal(a[n][:, cols], ref[n].astype(a[n].dtype), err_msg=f"{what}: {n}")
    np.testing.assert_array_equal(a["done"][:, cols], ref["done"].astype(a["done"].dtype), err_msg=f"{what}: done")
    np.testing.assert_array_equal(a["ep_return"][:, cols], ref["ep_return"], err_msg=f"{what}: ep_return")
    np.testing.assert_array_equal(a["ep_len"][:, cols], ref["ep_len"].astype(a["ep_len"].dtype), err_msg=f"{what}: ep_len")
    np.testing.assert_array_equal(a["pos"][:, :, cols], ref["pos"], err_msg=f"{what}: positions")
    K = ref["obs"].shape[1]
    np.testing.assert_array_equal(a["reset_obs"][:, cols].reshape(K, len(cols), -1), ref["reset_obs"],
                                  err_msg=f"{what}: reset obs")
    g = a["obs"][:, :, cols].reshape(ref["obs"].shape)
    f = a["final_obs"][:, :, cols].reshape(ref["final_obs"].shape)
    for t in range(ref["obs"].shape[0]):
        np.testing.assert_array_equal(g[t], ref["obs"][t], err_msg=f"{what}: obs at step {t}")
        d = ref["done"][t].astype(bool)
        np.testing.assert_array_equal(f[t][:, d], ref["final_obs"][t][:, d], err_msg=f"{what}: final obs at step {t}")


def test_c5_last_shard_slice_matches_oracle(c5_run):
    sel, host, done, ret, ep_len, scores, capped = c5_run
    sc = S.builtin("grid32")
    cols = np.arange(SLICE)
    ref = _oracle_replay(sc, OFF5 + SLICE0, host["act"][:, cols])
    _check_c5(host, cols, ref, f"global envs [{OFF5 + SLICE0}, {OFF5 + SLICE0 + SLICE})")
    assert ref["done"].sum() > 0 and ref["term"].sum() > 0


def test_c5_last_shard_capped_envs_match_oracle(c5_run):
    sel, host, done, ret, ep_len, scores, capped = c5_run
    assert len(capped) > 0, "no episode reached the 150-step cap"
    sc = S.builtin("grid32")
    for j, g in enumerate(capped):
        col = np.array([SLICE + j])
        ref = _oracle_replay(sc, OFF5 + int(g), host["act"][:, col])
        assert ((ref["ep_len"][:, 0] == CAP) & (ref["done"][:, 0] != 0)).any()
        _check_c5(host, col, ref, f"capped env {OFF5 + int(g)}")


def test_c5_gathered_returns_in_reference_order(c5_run):
    """All 65,536 envs: the gathered completed-episode list == every step's done envs' returns,
    step by step, then by global env id (completed_episode_scores of maddpg/agent.py:229-247)."""
    sel, host, done, ret, ep_len, scores, capped = c5_run
    want = np.concatenate([ret[t][done[t] != 0] for t in range(done.shape[0])])
    assert len(want) > 10_000
    np.testing.assert_array_equal(scores, want)


# ------------------------------------------------------------------------------------------ C2
E2, WARM2, GRAPH2, REPLAYS2 = 4096, 5, 16, 10


def test_c2_graph_replay_mode_matches_oracle():
    from marlnav.parallel import ReturnGather
    mp = pytest.MonkeyPatch()
    mp.delenv("GW_KERNEL", raising=False)
    try:
        env = VecGridEnv("grid32", num_envs=E2, fear=False, fear_weight=-2.0, max_steps=CAP, auto_reset=True,
                         seed=SEED, env_offset=0, stats=True)
    finally:
        mp.undo()
    assert env.kernel_path == "merged"
    dev = env.device
    gather = ReturnGather(E2, 0, 1, dev, window=GRAPH2)
    acc = torch.zeros_like(env.out["stats"])
    env.set_obs_async(True)
    env.reset()
    win_done, win_ret, pos_at = [], [], []
    for i in range(WARM2):  # bench.py's eager warmup steps
        into = gather.into()
        into["stats_acc"] = acc
        r = env.step(into=into)
        win_done.append(r.done.clone())
        win_ret.append(r.ep_return.clone())
        gather.push()
    gather.compact()
    graph = env.capture_steps(GRAPH2, gather)
    for rep in range(REPLAYS2):
        graph.replay()
        recv = gather._recv[:GRAPH2, 0]  # the window's slots stay readable until the next replay
        win_ret.append(recv[:, : 8 * E2].contiguous().view(torch.float64).reshape(GRAPH2, E2).clone())
        win_done.append(recv[:, 8 * E2: 9 * E2].clone())
        pos_at.append(env.state()["pos"].clone())
    env.obs_fence()
    # the last step's outputs (the captured steps write ep_return / done into the gather only)
    last = {n: env.out[n].clone() for n in ("reward", "term", "trunc", "mask", "crashes", "apples", "ep_len")}
    obs_final = env.out["obs"].clone()
    scores = gather.completed()
    torch.cuda.synchronize()
    done_g = torch.cat([torch.stack(win_done[:WARM2]).to(torch.uint8)] + [d for d in win_done[WARM2:]]).cpu().numpy()
    ret_g = torch.cat([torch.stack(win_ret[:WARM2])] + win_ret[WARM2:]).cpu().numpy()
    env.close()

    sc = S.builtin("grid32")
    T = WARM2 + GRAPH2 * REPLAYS2
    orc = O.OracleEnvs(sc, E2, fear=False, fear_weight=-2.0, max_steps=CAP, seed=SEED, reset=False)
    obs = np.zeros((sc.K, E2, sc.HW), np.float32)
    orc.reset_all(obs=obs, nthreads=16)
    outs = (O.StepOut * E2)()
    want_scores = []
    for t in range(T):
        orc.vec_step(None, obs=obs, outs=outs, nthreads=16)
        d = np.array([outs[e].done for e in range(E2)], np.uint8)
        rr = np.array([outs[e].ep_return for e in range(E2)])
        np.testing.assert_array_equal(done_g[t], d, err_msg=f"done at step {t}")
        np.testing.assert_array_equal(ret_g[t], rr, err_msg=f"ep_return at step {t}")
        want_scores.extend(rr[d != 0].tolist())
        if t >= WARM2 and (t - WARM2) % GRAPH2 == GRAPH2 - 1:
            rep = (t - WARM2) // GRAPH2
            np.testing.assert_array_equal(pos_at[rep].t().cpu().numpy(), orc.positions(),
                                          err_msg=f"positions after replay {rep}")
    K = sc.K
    o = [outs[e] for e in range(E2)]
    np.testing.assert_array_equal(last["reward"].cpu().numpy(), np.array([list(x.reward)[:K] for x in o]))
    np.testing.assert_array_equal(last["term"].cpu().numpy(), np.array([list(x.term)[:K] for x in o], np.uint8))
    np.testing.assert_array_equal(last["trunc"].cpu().numpy(), np.array([list(x.trunc)[:K] for x in o], np.uint8))
    np.testing.assert_array_equal(last["mask"].cpu().numpy().astype(np.uint16),
                                  np.array([list(x.mask)[:K] for x in o], np.uint16))
    np.testing.assert_array_equal(last["crashes"].cpu().numpy(), np.array([x.crashes for x in o]))
    np.testing.assert_array_equal(last["apples"].cpu().numpy(), np.array([x.apples_caught for x in o]))
    np.testing.assert_array_equal(last["ep_len"].cpu().numpy(), np.array([x.ep_len for x in o]))
    np.testing.assert_array_equal(obs_final.reshape(K, E2, -1).cpu().numpy(), obs, err_msg="final obs")
    np.testing.assert_array_equal(scores, np.array(want_scores))
    assert len(want_scores) > 1000
