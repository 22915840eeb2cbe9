"""HIP path vs the reference (golden trajectories) and vs the C oracle (native-RNG mode).

All tests here run the product path: libgridenv.so's kernels through the C ABI
(marlnav/_lib.py ctypes), on a real MI355X.  The oracle is only the checker.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

from _replay import load, load_single, replay, replay_single, single_cases

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCEN_OF = {"level3": "level3", "level3like": "level3", "grid32": "grid32", "grid64n8": "grid64_n8"}


def scenario_for(fname):
    return S.builtin(SCEN_OF[fname[len("traj_"):].rsplit("_", 1)[0]])


class GpuStepper:
    def __init__(self, sc, fear, weight, variant=0):
        self.env = VecGridEnv(sc, num_envs=1, fear=fear, fear_weight=weight, max_steps=150,
                              auto_reset=True, final_obs=True, debug=True, variant=variant)
        self.K, self.N = sc.K, sc.N

    def reset(self, spawn):
        obs, mask = self.env.reset(spawn=torch.as_tensor(np.asarray(spawn, np.int32)).view(1, -1))
        return obs[:, 0].cpu().numpy().reshape(self.K, -1), mask[0].cpu().numpy().astype(np.uint16)

    def step(self, rl, scripted, spawn_next):
        sp = None if spawn_next is None else np.asarray(spawn_next, np.int32).reshape(1, -1)
        r = self.env.step(np.asarray(rl, np.int32).reshape(1, -1), np.asarray(scripted, np.int32).reshape(1, -1), sp)
        torch.cuda.synchronize()
        g = lambda t: t[0].cpu().numpy()
        return dict(act=g(r.actions), mdr=g(r.mdr), final_pos=g(r.final_pos), crash_bits=int(g(r.crash_bits)),
                    restr_bits=int(g(r.restr_bits)), reward=g(r.reward), fear=g(r.fear), shaped=g(r.shaped),
                    term=g(r.term), trunc=g(r.trunc), crashes=int(g(r.crashes)), apples=int(g(r.apples)),
                    done=int(g(r.done)), ep_return=float(g(r.ep_return)), ep_fear=float(g(r.ep_fear)),
                    ep_len=int(g(r.ep_len)), obs=r.obs[:, 0].cpu().numpy().reshape(self.K, -1),
                    final_obs=r.final_obs[:, 0].cpu().numpy().reshape(self.K, -1),
                    mask=g(r.mask).astype(np.uint16))


@pytest.mark.parametrize("tag", single_cases(GOLD))
def test_gpu_replays_single_agent_trajectory(tag, kernel_path):
    """custom/customenv.py (single-agent CustomEnv) trajectories from the reference, bit-exact
    through the C ABI on every kernel path."""
    d = load_single(GOLD, tag)
    st = GpuStepper(S.builtin("level3_single"), tag.startswith("fear"), 0.0, variant=1)
    assert replay_single(st, d) == len(d["rl"])
    st.env.close()


def traj_cases():
    cases = []
    for path in sorted(glob.glob(os.path.join(GOLD, "traj_*.npz"))):
        z = np.load(path)
        for s in z["seeds"]:
            cases.append((os.path.basename(path), int(s)))
    return cases


@pytest.mark.parametrize("fname,seed", traj_cases())
def test_gpu_replays_reference_trajectory(fname, seed):
    d, meta = load(os.path.join(GOLD, fname), seed)
    sc = scenario_for(fname)
    st = GpuStepper(sc, bool(meta["fear"]), float(meta["fear_weight"]))
    T, err = replay(st, d, sc.K, sc.N)
    assert T > 0 and err == 0.0
    st.env.close()


def _compare_native(sc, E, fear, steps, nthreads=16, offset=0, seed=7, weight=-5.0, max_steps=150,
                    return_capped=False):
    """GPU native-RNG rollout == C oracle rollout, every output, every step (bit-exact).
    Returns the number of completed episodes (and, with return_capped, how many of them ended
    at the max_steps cap, maddpg/agent.py:243-247)."""
    env = VecGridEnv(sc, num_envs=E, fear=fear, fear_weight=weight, max_steps=max_steps, auto_reset=True,
                     seed=seed, env_offset=offset, final_obs=True, debug=True, stats=True)
    guard = torch.full((1 << 16,), 7.0, dtype=torch.float64, device=env.device)  # canary after stats
    orc = O.OracleEnvs(sc, E, fear=fear, fear_weight=weight, max_steps=max_steps, seed=seed, env_offset=offset,
                       reset=False)
    obs_o = np.zeros((sc.K, E, sc.HW), np.float32)
    orc.reset_all(obs=obs_o, nthreads=nthreads)
    obs_g, _ = env.reset()
    np.testing.assert_array_equal(obs_g.reshape(sc.K, E, -1).cpu().numpy(), obs_o, err_msg="reset obs")
    outs = (O.StepOut * E)()
    fin_o = np.zeros((sc.K, E, sc.HW), np.float32)
    done_total = capped = 0
    for t in range(steps):
        r = env.step()
        orc.vec_step(None, obs=obs_o, outs=outs, nthreads=nthreads, final_obs=fin_o)
        torch.cuda.synchronize()
        K, N = sc.K, sc.N
        get = lambda name, n: np.array([list(getattr(outs[e], name))[:n] for e in range(E)])
        np.testing.assert_array_equal(r.actions.cpu().numpy(), get("actions", N), err_msg=f"t={t} actions")
        np.testing.assert_array_equal(r.final_pos.cpu().numpy(), get("final_pos", N), err_msg=f"t={t} pos")
        np.testing.assert_array_equal(r.crash_bits.cpu().numpy(), np.array([outs[e].crash_bits for e in range(E)]), err_msg=f"t={t} crash")
        np.testing.assert_array_equal(r.reward.cpu().numpy(), get("reward", K), err_msg=f"t={t} reward")
        np.testing.assert_array_equal(r.fear.cpu().numpy(), get("fear", K), err_msg=f"t={t} fear")
        np.testing.assert_array_equal(r.shaped.cpu().numpy(), get("shaped", K), err_msg=f"t={t} shaped")
        np.testing.assert_array_equal(r.term.cpu().numpy(), get("term", K), err_msg=f"t={t} term")
        np.testing.assert_array_equal(r.trunc.cpu().numpy(), get("trunc", K), err_msg=f"t={t} trunc")
        dn = np.array([outs[e].done for e in range(E)])
        np.testing.assert_array_equal(r.done.cpu().numpy(), dn, err_msg=f"t={t} done")
        np.testing.assert_array_equal(r.ep_return.cpu().numpy(), np.array([outs[e].ep_return for e in range(E)]), err_msg=f"t={t} ret")
        np.testing.assert_array_equal(r.mask.cpu().numpy().astype(np.uint16), get("mask", K), err_msg=f"t={t} mask")
        np.testing.assert_array_equal(r.obs.reshape(K, E, -1).cpu().numpy(), obs_o, err_msg=f"t={t} obs")
        ep_len = np.array([outs[e].ep_len for e in range(E)])
        np.testing.assert_array_equal(r.ep_len.cpu().numpy(), ep_len, err_msg=f"t={t} ep_len")
        np.testing.assert_array_equal(r.ep_fear.cpu().numpy(), np.array([outs[e].ep_fear for e in range(E)]),
                                      err_msg=f"t={t} ep_fear")
        np.testing.assert_array_equal(r.apples.cpu().numpy(), np.array([outs[e].apples_caught for e in range(E)]),
                                      err_msg=f"t={t} apples")
        ended = np.flatnonzero(dn)  # terminal obs of the envs that ended (their next_state)
        np.testing.assert_array_equal(r.final_obs.reshape(K, E, -1)[:, ended].cpu().numpy(), fin_o[:, ended],
                                      err_msg=f"t={t} final_obs")
        capped += int(((dn != 0) & (ep_len == max_steps)).sum())
        # per-block statistics == the same sums over the oracle's outputs
        st = r.stats.sum(0).cpu().numpy()
        assert st[7] == E and st[1] == dn.sum()
        assert st[3] == sum(outs[e].crashes for e in range(E))
        np.testing.assert_allclose(st[0], sum(outs[e].ep_return for e in range(E) if outs[e].done), rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(st[2], get("fear", K).sum(), rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(st[5], get("shaped", K).sum(), rtol=1e-12, atol=1e-9)
        assert st[4] == sum(outs[e].apples_caught for e in range(E))
        assert st[6] == sum(outs[e].ep_len for e in range(E) if outs[e].done)
        done_total += int(dn.sum())
    assert bool((guard == 7.0).all()), "write past the stats buffer"
    env.close()
    return (done_total, capped) if return_capped else done_total


KERNEL_PATHS = {
    # the two kernel paths gw_create picks (round 6: the A/B-only paths v1 / split / fused and
    # the env-chunk pipelines were deleted)
    "defer": {"GW_KERNEL": "defer"},   # FeAR on: step_v2 <DEFER>, fear_v2 on a 2nd stream || obs_kernel
    "defer_narrow": {"GW_KERNEL": "defer", "GW_FEAR_BE": "narrow"},  # fear_v2 blocks of the bf16 obs default
    "merged": {"GW_KERNEL": "merged"},  # synchronous: step_v2 with FeAR inline, then obs_kernel
}


@pytest.fixture(params=sorted(KERNEL_PATHS))
def kernel_path(request, monkeypatch):
    """Every kernel path must pass the same bit-exact checks (selected by env vars read at
    gw_create)."""
    for k, v in KERNEL_PATHS[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


@pytest.mark.parametrize("name,fear", [("level3", False), ("level3", True), ("grid32", False), ("grid32", True),
                                       ("grid64_n8", False), ("grid64_n8", True)])
def test_native_rng_matches_oracle(name, fear, kernel_path):
    sc = S.builtin(name)
    E = 2048 if not fear else 512
    steps = 60 if not fear else 25
    done = _compare_native(sc, E, fear, steps)
    assert done > 0


def test_many_agents_k_gt_2_matches_oracle(kernel_path):
    """K > 2 RL agents (the KMAX = N kernel variants) on an open 8x8 map with N = 5."""
    sc = S.compile_scenario(S.level3_like(10, 16, 5, 3))
    _compare_native(sc, 512, True, 20)
    _compare_native(sc, 1024, False, 40)


@pytest.mark.parametrize("max_steps,steps,E", [(8, 40, 512), (150, 165, 192)])
def test_episode_cap_matches_oracle(max_steps, steps, E, kernel_path):
    """The TRAIN_STEPS cap (configs/custom_fear_5.yaml:5, maddpg/agent.py:243-247): episodes cut
    at max_steps are compared bit-exact (done, ep_len, ep_return, the terminal obs and the
    auto-reset obs after the cap), and some episodes do reach the cap."""
    sc = S.builtin("grid32")
    done, capped = _compare_native(sc, E, True, steps, max_steps=max_steps, seed=42, return_capped=True)
    assert done > 0 and capped > 0, (done, capped)


@pytest.mark.parametrize("E", [1, 77, 1000])
def test_ragged_env_counts_match_oracle(E, kernel_path):
    """E not a multiple of any block size (partial last blocks of step_v2, fear_v2, obs_kernel)
    and a non-zero global env offset."""
    _compare_native(S.builtin("grid32"), E, True, 12, offset=12345)
    _compare_native(S.builtin("level3"), E, False, 12, offset=7)


def test_sharding_is_invariant():
    """Two shards (env_offset 0 and E/2) reproduce the single-device run env for env."""
    sc = S.builtin("grid32")
    E = 4096
    full = VecGridEnv(sc, num_envs=E, fear=True, seed=3, debug=True)
    a = VecGridEnv(sc, num_envs=E // 2, fear=True, seed=3, env_offset=0, debug=True)
    b = VecGridEnv(sc, num_envs=E // 2, fear=True, seed=3, env_offset=E // 2, debug=True)
    for env in (full, a, b):
        env.reset()
    for _ in range(30):
        rf, ra, rb = full.step(), a.step(), b.step()
        torch.cuda.synchronize()
        for name in ("final_pos", "reward", "fear", "done", "ep_return"):
            x = getattr(rf, name).cpu()
            y = torch.cat([getattr(ra, name).cpu(), getattr(rb, name).cpu()])
            assert torch.equal(x, y), name
        assert torch.equal(rf.obs.cpu(), torch.cat([ra.obs.cpu(), rb.obs.cpu()], dim=1))
    for env in (full, a, b):
        env.close()


@pytest.mark.parametrize("name,E", [("grid32", 65536), ("grid64_n8", 65536)])
def test_full_size_properties(name, E, kernel_path):
    """BASELINE sizes: size-independent invariants on every env + a bit-exact slice vs the oracle."""
    sc = S.builtin(name)
    env = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, seed=9, stats=True, debug=True)
    sl0, sl = 4096 + 128, 256  # a slice that straddles pipeline chunks and blocks
    orc = O.OracleEnvs(sc, sl, fear=True, fear_weight=-5.0, seed=9, env_offset=sl0, reset=False)
    obs_o = np.zeros((sc.K, sl, sc.HW), np.float32)
    orc.reset_all(obs=obs_o)
    env.reset()
    outs = (O.StepOut * sl)()
    road = torch.as_tensor(sc.region.astype(bool), device=env.device)
    for t in range(12):
        r = env.step()
        orc.vec_step(None, obs=obs_o, outs=outs, nthreads=16)
        pos = env.positions()                                        # [E, N] after any auto-reset
        srt = pos.sort(1).values
        assert bool((srt[:, 1:] != srt[:, :-1]).all()), "two agents share a cell"
        assert bool(road[pos.long()].all()), "agent off the road"
        # obs encodes exactly the agents: N cells per agent-obs carry agent values
        o = r.obs.reshape(sc.K, E, -1)
        agents_in_obs = ((o != 0) & (o != -1) & (o != 9)).sum(-1)
        assert bool((agents_in_obs == sc.N).all())
        st = r.stats.sum(0)
        assert float(st[7]) == E and float(st[1]) == float(r.done.sum())
        np.testing.assert_array_equal(r.final_pos[sl0:sl0 + sl].cpu().numpy(),
                                      np.array([list(outs[e].final_pos)[:sc.N] for e in range(sl)]))
        np.testing.assert_array_equal(r.ep_return[sl0:sl0 + sl].cpu().numpy(),
                                      np.array([outs[e].ep_return for e in range(sl)]))
        np.testing.assert_array_equal(o[:, sl0:sl0 + sl].cpu().numpy(), obs_o)
    env.close()


def _map_scenario(region2d, N):
    """A compiled scenario of a golden map (single policy, MdR stay) with N world agents."""
    H, W = region2d.shape
    road = np.argwhere(region2d == 1)[0]
    full = {"slicex": [0, H, 0], "slicey": [0, W, 0]}
    return S.compile_scenario({
        "AgentLocations": [], "Map": {"Region": region2d.tolist(), "Walls": [], "OneWays": []},
        "MdRs": {"00": dict(mdr=0, **full)}, "N_Agents": N, "N_Intelligent": 1,
        "Policies": {"00": dict(directionWeights=[1, 1, 1, 1], stepWeights=[1, 1, 0], **full)},
        "SpecificAction4Agents": [], "defaultAction": "random", "Apples": {"apple_0": [int(road[0]), int(road[1])]}})


@pytest.mark.parametrize("name", ["level3", "grid32", "open6_n8", "open6_n3", "open5x8_n5"])
def test_gpu_fear_matrix_and_feal_match_reference(name):
    """gw_fear_matrix == Responsibility.FeAR / FeAL golden vectors from the reference, every case
    bit-exact, all cases of a map in one launch."""
    z = np.load(os.path.join(GOLD, "fear_matrix.npz"))
    d = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(name + "/")}
    N = d["loc"].shape[1]
    env = VecGridEnv(_map_scenario(d["region"], N), num_envs=1, fear=True)
    bits = (d["in_list"].astype(np.int64) << np.arange(N)).sum(1)
    o = env.fear_matrix(d["loc"], d["act"], d["mdr"], bits)
    torch.cuda.synchronize()
    for k in ("vm", "va", "resp", "feal_vm", "feal_va", "feal"):
        np.testing.assert_array_equal(o[k].cpu().numpy(), d[k], err_msg=f"{name} {k}")
    env.close()


def test_gpu_fear_matrix_row_equals_step_fear():
    """Row k of the full matrix for the env's close-agent list reproduces the per-step FeAR of
    RL agent k (ma_customenv.py:247-252), on live states of a native-RNG rollout."""
    sc = S.builtin("grid32")
    E = 1024
    env = VecGridEnv(sc, num_envs=E, fear=True, seed=4, debug=True)
    env.reset()
    for _ in range(5):
        pos = env.positions()
        r = env.step()
        torch.cuda.synchronize()
        act, mdr = r.actions.clone(), r.mdr.clone()
        for k in range(sc.K):
            rr, cc = pos // sc.W, pos % sc.W
            dist = (rr - rr[:, k:k + 1]).abs() + (cc - cc[:, k:k + 1]).abs()
            in_list = ((dist <= 5).to(torch.int64) << torch.arange(sc.N, device=pos.device)).sum(1)
            o = env.fear_matrix(pos, act, mdr, in_list)
            row = o["resp"][:, k, :].cpu().numpy()
            want = r.fear[:, k].cpu().numpy()
            got = np.array([np.sum(np.pad(row[e][None], ((k, sc.N - 1 - k), (0, 0)))) for e in range(E)])
            np.testing.assert_array_equal(got, want)
    env.close()
