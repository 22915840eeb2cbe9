"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE Python itself.

Runs only in the build container, where the read-only reference checkout lives at
/root/reference (it never travels to the GPU box).  The reference env imports pettingzoo,
gymnasium and pygame, none of which is installed; inert stand-ins (a ParallelEnv base with a
``num_agents`` property, Discrete/Box holders, an empty pygame module) are placed in
sys.modules first.  Rendering stays off, nothing else of the reference is replaced.

Fixtures written (all inputs + the reference's outputs):
  maps.npz         compiled Level-3 maps as CustomMAEnv holds them (+ the policy vectors)
  transition.npz   GWorld.UpdateGWorld known-answer tests     (custom/grid_world.py:424-563)
  fear.npz         Responsibility.FeAR_4_one_actor KATs      (custom/Responsibility.py:135-210)
  traj_*.npz       CustomMAEnv trajectories in replay form    (custom/ma_customenv.py:169-334)
                   + the rollout arithmetic of maddpg/agent.py:124-173

usage:  python tests/golden/make_golden.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import tempfile
import time
import types

import numpy as np

REF = os.environ.get("MARLNAV_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(OUT))
sys.path.insert(0, os.path.join(REPO, "marl-responsible-nav_amd"))
from marlnav import scenario as S  # noqa: E402  (the input definitions only)


def install_stubs():
    class ParallelEnv:
        @property
        def num_agents(self):
            return len(self.agents)

    pz = types.ModuleType("pettingzoo")
    pz.ParallelEnv = ParallelEnv
    pz.AECEnv = object
    pzu = types.ModuleType("pettingzoo.utils")
    pzu.agent_selector = object

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low, high, shape, dtype):
            self.shape = shape

    class Env:  # gymnasium.Env base of the single-agent CustomEnv (customenv.py:45)
        pass

    gym = types.ModuleType("gymnasium")
    gym.Env = Env
    sp = types.ModuleType("gymnasium.spaces")
    sp.Discrete, sp.Box, gym.spaces = Discrete, Box, sp
    for k, v in {"pettingzoo": pz, "pettingzoo.utils": pzu, "gymnasium": gym,
                 "gymnasium.spaces": sp, "pygame": types.ModuleType("pygame")}.items():
        sys.modules.setdefault(k, v)


def import_reference():
    install_stubs()
    sys.dont_write_bytecode = True
    os.chdir(REF)
    # /root/reference/custom is a namespace package (no __init__.py): a regular package of the
    # same name anywhere on sys.path (this repo's CustomMAEnv facade) would shadow it
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != os.path.join(REPO, "marl-responsible-nav_amd")]
    sys.path.insert(0, REF)
    import custom.grid_world as G
    import custom.custom_agent as CA
    import custom.Responsibility as R
    import custom.ma_customenv as M
    return G, CA, R, M


def cell(W, loc):
    return int(loc[0]) * W + int(loc[1])


# ----------------------------------------------------------------------------------------
def make_world(G, CA, region2d, locs_rc):
    world = G.GWorld(np.array(region2d), Walls=[], OneWays=[])
    for r, c in locs_rc:
        ok = world.AddAgent(CA.CustomAgent(), (int(r), int(c)), printStatus=False)
        assert ok
    return world


def clustered_positions(rng, region2d, N, radius):
    H, W = region2d.shape
    road = np.argwhere(region2d == 1)
    center = road[rng.integers(len(road))]
    d = np.abs(road - center).sum(1)
    pool = road[d <= radius]
    if len(pool) < N:
        pool = road
    idx = rng.choice(len(pool), N, replace=False)
    return [tuple(map(int, p)) for p in pool[idx]]


def gen_transition(G, CA, maps, rng, quick):
    out = {}
    for name, (region2d, N, K, cases) in maps.items():
        if quick:
            cases = min(cases, 200)
        H, W = region2d.shape
        L = np.zeros((cases, N), np.int32)
        A = np.zeros((cases, N), np.int32)
        AP = np.full((cases, K), -1, np.int32)
        CR = np.zeros((cases, N), np.uint8)
        RS = np.zeros((cases, N), np.uint8)
        FI = np.zeros((cases, N), np.int32)
        CA_ = np.full((cases, 4 * K * K, 2), -1, np.int32)
        NC = np.zeros(cases, np.int32)
        for i in range(cases):
            radius = int(rng.integers(1, 7))
            locs = clustered_positions(rng, region2d, N, radius)
            acts = rng.integers(0, 9, N)
            apples = {}
            for k in range(K):
                if rng.random() < 0.8:
                    pr = clustered_positions(rng, region2d, 1, 3)[0] if rng.random() < 0.5 else locs[int(rng.integers(N))]
                    apples[f"apple_{k}"] = (int(pr[0]), int(pr[1]))
                    AP[i, k] = cell(W, pr)
            world = make_world(G, CA, region2d, locs)
            ret = world.UpdateGWorld(ActionID4Agents=[(n, int(acts[n])) for n in range(N)],
                                     apples=apples, apple_eaters=list(range(K)))
            crashes, restr, _, caught = ret
            L[i] = [cell(W, p) for p in locs]
            A[i] = acts
            CR[i] = np.array(crashes, np.uint8)
            RS[i] = np.array(restr, np.uint8)
            FI[i] = [cell(W, p) for p in world.AgentLocations]
            NC[i] = len(caught)
            for j, (agent, akey) in enumerate(caught):
                CA_[i, j] = (agent, int(akey[-1]))
        out[name] = dict(region=region2d.astype(np.uint8), loc=L, act=A, apples=AP, crash=CR,
                         restricted=RS, final=FI, caught=CA_, n_caught=NC)
    return out


def crafted_transition(G, CA):
    """The hand-checked cases of SURVEY.md Appendix A on an open 5x8 map (+ more)."""
    region = np.ones((5, 8))
    cases = [
        ([(2, 2)], [4]),                       # N=1: never moves
        ([(0, 1), (0, 2)], [4, 4]),            # follow-through, same direction
        ([(0, 1), (0, 3)], [4, 3]),            # head-on into the same cell
        ([(0, 1), (0, 2)], [4, 3]),            # swap
        ([(0, 1), (0, 3)], [8, 0]),            # Right2 into a stationary agent
        ([(0, 0), (0, 2)], [8, 4]),            # 2-step behind a 1-step, same direction
        ([(0, 0), (0, 1)], [8, 8]),            # 2-step follow-through
        ([(1, 1), (1, 2), (1, 3)], [4, 4, 4]), # train of three
        ([(1, 1), (1, 2), (1, 3)], [4, 4, 3]), # cascade after revert
        ([(2, 0), (2, 2), (0, 1)], [8, 3, 6]), # crossing paths
        ([(4, 7), (0, 0)], [6, 5]),            # edge clipping (restricted)
        ([(1, 0), (3, 0), (2, 1)], [6, 5, 3]), # three-way
    ]
    out = []
    for locs, acts in cases:
        world = make_world(G, CA, region, locs)
        crashes, restr = world.UpdateGWorld(ActionID4Agents=list(enumerate(acts)))
        out.append(dict(loc=[cell(8, p) for p in locs], act=acts, crash=[int(x) for x in crashes],
                        restricted=[int(x) for x in restr],
                        final=[cell(8, p) for p in world.AgentLocations]))
    return out


def gen_fear(G, CA, R, maps, rng, quick):
    out = {}
    for name, (region2d, mdr_cells, N, K, cases) in maps.items():
        if quick:
            cases = min(cases, 60)
        H, W = region2d.shape
        LOC = np.zeros((cases, N), np.int32)
        ACT = np.zeros((cases, N), np.int32)
        MDR = np.zeros((cases, N), np.int32)
        ACTOR = np.zeros(cases, np.int32)
        LIST = np.zeros((cases, N), np.uint8)
        RESP = np.zeros((cases, N, N), np.float64)
        VM = np.zeros((cases, N, N), np.int32)
        VA = np.zeros((cases, N, N), np.int32)
        SUM = np.zeros(cases, np.float64)
        for i in range(cases):
            radius = int(rng.integers(2, 9))
            locs = clustered_positions(rng, region2d, N, radius)
            acts = rng.integers(0, 9, N)
            mdr = np.array([mdr_cells[cell(W, p)] for p in locs]) if rng.random() < 0.5 else rng.integers(0, 9, N)
            actor = int(rng.integers(0, K))
            if rng.random() < 0.1:
                acts[actor] = mdr[actor]
            in_list = [n == actor or (abs(locs[n][0] - locs[actor][0]) + abs(locs[n][1] - locs[actor][1])) <= 5
                       for n in range(N)]
            agents = [(n, int(acts[n])) for n in range(N) if in_list[n]]
            world = make_world(G, CA, region2d, locs)
            resp, vm, va, _, _ = R.FeAR_4_one_actor(world, agents, [[n, int(mdr[n])] for n in range(N)], actor)
            LOC[i] = [cell(W, p) for p in locs]
            ACT[i] = acts
            MDR[i] = mdr
            ACTOR[i] = actor
            LIST[i] = in_list
            RESP[i] = resp
            VM[i] = vm
            VA[i] = va
            SUM[i] = np.sum(resp)
        R.CountValidMovesOfAffected_tuple.cache_clear()
        out[name] = dict(region=region2d.astype(np.uint8), loc=LOC, act=ACT, mdr=MDR, actor=ACTOR,
                         in_list=LIST, resp=RESP, vm=VM, va=VA, sum=SUM)
    return out


# ----------------------------------------------------------------------------------------
def make_env_factory(G, M, sc_dict, name):
    """CustomMAEnv on a (possibly synthetic) scenario: patch the module globals that
    ma_customenv.py reads (Scenario :27, total_num_agents :28, N_INTELLIGENT_AGENTS :19) and
    override the hard-coded apples of setup_env (:422)."""
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump({name: sc_dict}, f)
        path = f.name
    ref_sc = G.LoadJsonScenario(json_filename=path, scenario_name=name)
    os.unlink(path)
    N, K = sc_dict["N_Agents"], sc_dict["N_Intelligent"]
    apples = {k: tuple(v) for k, v in sc_dict["Apples"].items()}

    class Env(M.CustomMAEnv):
        def setup_env(self):
            super().setup_env()
            self.apples = dict(apples)

    def factory(fear, seed):
        M.Scenario = ref_sc
        M.total_num_agents = N
        M.N_INTELLIGENT_AGENTS = K
        return Env(render=False, fear=fear, seed=seed)

    return factory


def run_traj(factory, W, N, K, fear, fear_weight, seed, steps, policy, max_steps=150):
    random.seed(seed)
    np.random.seed(seed)
    env = factory(fear, seed)
    HW = None
    rng = np.random.default_rng(1000 + seed)
    rec = {k: [] for k in ["rl", "act", "mdr", "pos", "reward", "fear", "shaped", "term", "trunc",
                           "crash_bits", "restr_bits", "crashes", "apples", "obs", "mask", "done",
                           "ep_return", "ep_fear", "ep_len", "reset_pos", "reset_obs", "reset_mask",
                           "reset_at"]}
    obs, info = env.reset()

    def rec_reset(step_idx):
        rec["reset_at"].append(step_idx)
        rec["reset_pos"].append([cell(W, p) for p in env.World.AgentLocations])
        rec["reset_obs"].append(np.stack([np.round(obs[f"agent_{k}"] * 2) for k in range(K)]).astype(np.int8))
        rec["reset_mask"].append([int(np.dot(info[f"agent_{k}"]["action_mask"], 1 << np.arange(9))) for k in range(K)])

    rec_reset(-1)
    score = 0.0
    fear_score = 0.0
    ep_len = 0
    for t in range(steps):
        if policy == "uniform":
            a = rng.integers(0, 9, K)
        else:
            a = np.array([rng.choice(np.flatnonzero(info[f"agent_{k}"]["action_mask"])) for k in range(K)])
        obs, reward, term, trunc, info = env.step(tuple(int(x) for x in a))
        ep_len += 1
        FeAR = info["fear"]
        # maddpg/agent.py:124-141,173
        shaped = {ag: fear_weight * FeAR[ag] + reward[ag] for ag in reward.keys()}
        shaped_arr = np.array(list(shaped.values()))
        fear_sum = np.sum(list(FeAR.values()))
        fear_score += fear_sum
        score += np.sum(np.array(list(shaped.values())).transpose(), axis=-1)
        rec["rl"].append(a)
        rec["act"].append([int(x[1]) for x in env.Action4Agents])
        rec["mdr"].append([int(x[1]) for x in env.MdR4Agents])
        rec["pos"].append([cell(W, p) for p in env.World.AgentLocations])
        rec["reward"].append([reward[f"agent_{k}"] for k in range(K)])
        rec["fear"].append([float(FeAR[f"agent_{k}"]) for k in range(K)])
        rec["shaped"].append(shaped_arr)
        rec["term"].append([term[f"agent_{k}"] for k in range(K)])
        rec["trunc"].append([trunc[f"agent_{k}"] for k in range(K)])
        rec["crash_bits"].append(sum(int(bool(c)) << n for n, c in enumerate(env.World.AgentCrash)))
        rec["restr_bits"].append(sum(int(bool(c)) << n for n, c in enumerate(env.World.RestrictedMove)))
        rec["crashes"].append(info["agent_crashes"])
        rec["apples"].append(info["apples_caught"])
        rec["obs"].append(np.stack([np.round(obs[f"agent_{k}"] * 2) for k in range(K)]).astype(np.int8))
        rec["mask"].append([int(np.dot(info[f"agent_{k}"]["action_mask"], 1 << np.arange(9))) for k in range(K)])
        done = all(term.values()) or all(trunc.values()) or ep_len >= max_steps
        rec["done"].append(done)
        rec["ep_return"].append(score)
        rec["ep_fear"].append(fear_score)
        rec["ep_len"].append(ep_len)
        if done:
            obs, info = env.reset()
            rec_reset(t)
            score, fear_score, ep_len = 0.0, 0.0, 0
    out = {}
    for k, v in rec.items():
        out[k] = np.array(v)
    out["rl"] = out["rl"].astype(np.int32)
    out["act"] = out["act"].astype(np.int32)
    out["mdr"] = out["mdr"].astype(np.int32)
    out["pos"] = out["pos"].astype(np.int32)
    out["reward"] = out["reward"].astype(np.float64)
    out["term"] = out["term"].astype(np.uint8)
    out["trunc"] = out["trunc"].astype(np.uint8)
    out["done"] = out["done"].astype(np.uint8)
    out["reset_pos"] = out["reset_pos"].astype(np.int32)
    out["reset_at"] = out["reset_at"].astype(np.int32)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    t0 = time.time()
    G, CA, R, M = import_reference()
    rng = np.random.default_rng(20241101)

    # ---- maps (Level 3 as the reference compiles it) ----
    env = M.CustomMAEnv(render=False, fear=False, seed=0)
    env.reset()
    pol = {}
    for key, v in env.policies.items():
        pol[key] = np.stack([CA.GeneratePolicy(StepWeights=v["stepWeights"], DirectionWeights=v["directionWeights"]),
                             CA.GeneratePolicy(StepWeights=v["stepWeights"], DirectionWeights=None)])
    mdr_act = np.array([[env.mdrs[str(env.mdr_map[r, c]).zfill(2)]["mdr"] for c in range(16)] for r in range(10)])
    np.savez_compressed(os.path.join(OUT, "maps.npz"), region=env.Region, policy_map=env.policy_map,
                        mdr_map=env.mdr_map, mdr_action=mdr_act, policy_keys=np.array(list(pol.keys())),
                        policy_p=np.stack(list(pol.values())), apples=np.array([[9, 0], [5, 10]]),
                        mask=np.array([[int(np.dot(env.get_action_mask(f"agent_{k}")["action_mask"], 1 << np.arange(9)))
                                        for k in range(2)]]))
    print("maps done", time.time() - t0)

    # ---- scenarios for the synthetic configs ----
    sc32 = S.level3_like(32, 32, 4, 2)
    sc64 = S.level3_like(64, 64, 8, 2)
    lvl3 = S.level3_like(10, 16, 4, 2)
    reg = {n: np.array(s["Map"]["Region"]) for n, s in [("level3", lvl3), ("grid32", sc32), ("grid64_n8", sc64)]}
    open6 = np.ones((6, 6))
    open5x8 = np.ones((5, 8))

    tr = gen_transition(G, CA, {
        "level3": (np.array(env.Region), 4, 2, 4000),
        "grid32": (reg["grid32"], 4, 2, 1500),
        "grid64_n8": (reg["grid64_n8"], 8, 2, 1500),
        "open6_n8": (open6, 8, 2, 1500),
        "open6_n5": (open6, 5, 3, 800),
        "open5x8_n2": (open5x8, 2, 2, 500),
        "open5x8_n3": (open5x8, 3, 1, 500),
        "open5x8_n1": (open5x8, 1, 1, 50),
    }, rng, args.quick)
    flat = {}
    for name, d in tr.items():
        for k, v in d.items():
            flat[f"{name}/{k}"] = v
    crafted = crafted_transition(G, CA)
    flat["crafted_json"] = np.array(json.dumps(crafted))
    np.savez_compressed(os.path.join(OUT, "transition.npz"), **flat)
    print("transition done", time.time() - t0)

    c32 = S.compile_scenario(sc32)
    c64 = S.compile_scenario(sc64)
    c3 = S.compile_scenario(lvl3)
    fe = gen_fear(G, CA, R, {
        "level3": (np.array(env.Region), c3.mdr, 4, 2, 1200),
        "grid32": (reg["grid32"], c32.mdr, 4, 2, 400),
        "grid64_n8": (reg["grid64_n8"], c64.mdr, 8, 2, 250),
        "open6_n8": (open6, np.zeros(36, np.int32), 8, 2, 250),
        "open6_n3": (open6, np.zeros(36, np.int32), 3, 3, 300),
    }, rng, args.quick)
    flat = {}
    for name, d in fe.items():
        for k, v in d.items():
            flat[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(OUT, "fear.npz"), **flat)
    print("fear done", time.time() - t0)

    # ---- trajectories ----
    fac_l3 = make_env_factory(G, M, lvl3, "level3_like")
    # Level 3 itself, straight from the reference's own Scenarios.json
    ref_l3 = M.Scenario

    def fac_ref(fear, seed):
        M.Scenario = ref_l3
        M.total_num_agents = 4
        M.N_INTELLIGENT_AGENTS = 2
        return M.CustomMAEnv(render=False, fear=fear, seed=seed)

    fac_32 = make_env_factory(G, M, sc32, "grid32")
    fac_64 = make_env_factory(G, M, sc64, "grid64_n8")
    q = 4 if args.quick else 1
    plans = [
        ("traj_level3_nofear", fac_ref, 16, 4, 2, False, -2.0, [0, 1, 2, 3], 400 // q),
        ("traj_level3_fear", fac_ref, 16, 4, 2, True, -5.0, [0, 1, 2, 3], 120 // q),
        ("traj_level3like_fear", fac_l3, 16, 4, 2, True, -3.0, [5], 60 // q),
        ("traj_grid32_nofear", fac_32, 32, 4, 2, False, -5.0, [0, 1], 300 // q),
        ("traj_grid32_fear", fac_32, 32, 4, 2, True, -5.0, [0, 1], 80 // q),
        ("traj_grid64n8_nofear", fac_64, 64, 8, 2, False, -5.0, [0], 200 // q),
        ("traj_grid64n8_fear", fac_64, 64, 8, 2, True, -5.0, [3], 40 // q),
    ]
    for fname, fac, W, N, K, fear, wgt, seeds, steps in plans:
        flat = {"W": W, "N": N, "K": K, "fear": int(fear), "fear_weight": wgt}
        for s in seeds:
            d = run_traj(fac, W, N, K, fear, wgt, s, steps, "uniform" if s % 2 == 0 else "masked")
            for k, v in d.items():
                flat[f"s{s}/{k}"] = v
        flat["seeds"] = np.array(seeds)
        np.savez_compressed(os.path.join(OUT, f"{fname}.npz"), **flat)
        print(fname, "done", time.time() - t0)


if __name__ == "__main__":
    main()
