"""Golden trajectories of the single-agent variant ``custom/customenv.py`` (CustomEnv), generated
from the REFERENCE Python itself (build container only; /root/reference never travels).

Same harness as make_golden.py (inert pettingzoo/gymnasium/pygame stand-ins, rendering off).
The module's unseeded spawn generator ``rng`` (customenv.py:18) is replaced by a seeded one and
``random`` / ``np.random`` are seeded, so a run is reproducible; everything else is the
reference's code.  Recorded in replay form: spawns, all N actions after the RL override, and
the outputs of every step (obs, float reward, terminated, truncated, restricted, fear, episode
return/length).  Episodes are restarted on terminated / truncated or after 150 steps.

usage:  python tests/golden/make_golden_single.py
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import cell, import_reference  # noqa: E402


def run(CE, fear, seed, steps, policy, max_steps=150):
    random.seed(seed)
    np.random.seed(seed)
    CE.rng = np.random.default_rng(5000 + seed)
    env = CE.CustomEnv(render=False, fear=fear)
    W = 16
    act_rng = np.random.default_rng(7000 + seed)
    rec = {k: [] for k in ["rl", "act", "mdr", "pos", "reward", "fear", "term", "trunc", "restricted",
                           "crash_bits", "obs", "done", "ep_r", "ep_l", "reset_pos", "reset_obs", "reset_at"]}
    obs, _ = env.reset()

    def rec_reset(t):
        rec["reset_at"].append(t)
        rec["reset_pos"].append([cell(W, p) for p in env.World.AgentLocations])
        rec["reset_obs"].append(np.round(np.array(obs) * 2).astype(np.int8))

    rec_reset(-1)
    ep_len = 0
    for t in range(steps):
        if policy == "uniform":
            a = int(act_rng.integers(0, 9))
        else:  # destination on the road (get_action_mask semantics), to meet apple and agents more often
            r0, c0 = env.World.AgentLocations[0]
            ok = []
            for b in range(9):
                dr = sum(m[0] for m in CE.ActionMoves[b])
                dc = sum(m[1] for m in CE.ActionMoves[b])
                r1, c1 = r0 + dr, c0 + dc
                if 0 <= r1 < 10 and 0 <= c1 < 16 and env.Region[r1, c1] == 1:
                    ok.append(b)
            if policy == "seek" and act_rng.random() < 0.7:  # greedy towards the apple (9, 15)
                d = [abs(9 - r0 - sum(m[0] for m in CE.ActionMoves[b])) + abs(15 - c0 - sum(m[1] for m in CE.ActionMoves[b]))
                     for b in ok]
                a = int(ok[int(np.argmin(d))])
            else:
                a = int(act_rng.choice(ok))
        obs, reward, term, trunc, info = env.step([a])
        ep_len += 1
        rec["rl"].append(a)
        rec["act"].append([a] + env.World._last_actions[1:])
        rec["pos"].append([cell(W, p) for p in env.World.AgentLocations])
        rec["mdr"].append([int(m[1]) for m in env.MdR4Agents])
        rec["reward"].append(float(reward[0]))
        rec["fear"].append(float(info["fear"]))
        rec["term"].append(bool(term[0]))
        rec["trunc"].append(bool(trunc))
        rec["restricted"].append(bool(info["restricted"]))
        rec["crash_bits"].append(sum(int(bool(c)) << n for n, c in enumerate(env.World.AgentCrash)))
        rec["obs"].append(np.round(np.array(obs) * 2).astype(np.int8))
        rec["ep_r"].append(float(info["episode"]["r"]))
        rec["ep_l"].append(int(info["episode"]["l"]))
        done = bool(term[0]) or bool(trunc) or ep_len >= max_steps
        rec["done"].append(done)
        if done:
            obs, _ = env.reset()
            rec_reset(t)
            ep_len = 0
    out = {k: np.array(v) for k, v in rec.items()}
    for k in ("rl", "act", "mdr", "pos", "reset_pos", "reset_at"):
        out[k] = out[k].astype(np.int32)
    for k in ("term", "trunc", "restricted", "done"):
        out[k] = out[k].astype(np.uint8)
    return out


def main():
    G, CA, R, M = import_reference()
    import custom.customenv as CE
    # the scripted actions are not kept by the env: record what SelectActionsForAll returns
    orig = G.GWorld.SelectActionsForAll

    def select(self, *a, **k):
        acts = orig(self, *a, **k)
        self._last_actions = [int(x[1]) for x in acts]
        return acts

    G.GWorld.SelectActionsForAll = select
    flat = {}
    for fear, seed, steps, policy in [(True, 0, 300, "uniform"), (True, 1, 400, "valid"), (False, 2, 300, "valid"),
                                      (True, 3, 400, "valid"), (True, 4, 600, "seek"), (False, 5, 600, "seek")]:
        d = run(CE, fear, seed, steps, policy)
        for k, v in d.items():
            flat[f"{'fear' if fear else 'nofear'}_{seed}/{k}"] = v
    G.GWorld.SelectActionsForAll = orig
    np.savez_compressed(os.path.join(HERE, "single_traj.npz"), **flat)
    for k, v in flat.items():
        if k.endswith("/reward"):
            tag = k.split("/")[0]
            print(tag, "steps", v.shape[0], "episodes", flat[tag + "/reset_at"].shape[0] - 1,
                  "apples", int((v >= 10).sum()), "crashes", int(flat[tag + "/term"].sum()),
                  "bonus", int((np.abs(v - np.round(v)) > 1e-9).sum()), "fear!=0", int((flat[tag + "/fear"] != 0).sum()))


if __name__ == "__main__":
    main()
