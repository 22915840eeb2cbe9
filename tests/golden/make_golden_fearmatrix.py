"""Golden vectors of the full FeAR matrix and FeAL (custom/Responsibility.py:57-132, 213-303),
generated from the REFERENCE Python itself (build container only).

Each case: agent cells, the joint action list ActionID4Agents (agents absent from the list take
the 'stay' default and ignore swaps, as in the env's close_agents lists), per-agent MdR; outputs
Resp [N, N], ValidMoves_moveDeRigueur / _action [N, N], FeAL [N], its two ValidMoves vectors.

usage:  python tests/golden/make_golden_fearmatrix.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import S, cell, clustered_positions, import_reference, make_world  # noqa: E402


def gen(G, CA, R, region2d, mdr_cells, N, cases, rng):
    H, W = region2d.shape
    rec = {k: [] for k in ["loc", "act", "mdr", "in_list", "resp", "vm", "va", "feal", "feal_vm", "feal_va"]}
    for i in range(cases):
        locs = clustered_positions(rng, region2d, N, int(rng.integers(2, 9)))
        acts = rng.integers(0, 9, N)
        mdr = np.array([mdr_cells[cell(W, p)] for p in locs]) if rng.random() < 0.5 else rng.integers(0, 9, N)
        same = rng.random(N) < 0.15
        acts[same] = mdr[same]
        in_list = np.ones(N, bool) if rng.random() < 0.6 else rng.random(N) < 0.7
        agents = [(n, int(acts[n])) for n in range(N) if in_list[n]]
        mdr_list = [[n, int(mdr[n])] for n in range(N)]
        world = make_world(G, CA, region2d, locs)
        resp, vm, va, _, _ = R.FeAR(world, agents, mdr_list)
        world = make_world(G, CA, region2d, locs)
        feal, fvm, fva, _, _ = R.FeAL(world, agents, mdr_list)
        R.CountValidMovesOfAffected_tuple.cache_clear()
        rec["loc"].append([cell(W, p) for p in locs])
        rec["act"].append(acts)
        rec["mdr"].append(mdr)
        rec["in_list"].append(in_list)
        rec["resp"].append(resp)
        rec["vm"].append(vm)
        rec["va"].append(va)
        rec["feal"].append(feal)
        rec["feal_vm"].append(fvm)
        rec["feal_va"].append(fva)
    out = {k: np.array(v) for k, v in rec.items()}
    for k in ("loc", "act", "mdr", "vm", "va", "feal_vm", "feal_va"):
        out[k] = out[k].astype(np.int32)
    out["in_list"] = out["in_list"].astype(np.uint8)
    out["region"] = region2d.astype(np.uint8)
    return out


def main():
    G, CA, R, M = import_reference()
    rng = np.random.default_rng(20241117)
    lvl3 = S.compile_scenario(S.level3_like(10, 16, 4, 2))
    c32 = S.compile_scenario(S.level3_like(32, 32, 4, 2))
    maps = {
        "level3": (lvl3.region.reshape(10, 16), lvl3.mdr, 4, 240),
        "grid32": (c32.region.reshape(32, 32), c32.mdr, 4, 120),
        "open6_n8": (np.ones((6, 6)), np.zeros(36, np.int32), 8, 60),
        "open6_n3": (np.ones((6, 6)), np.zeros(36, np.int32), 3, 120),
        "open5x8_n5": (np.ones((5, 8)), np.zeros(40, np.int32), 5, 80),
    }
    flat = {}
    for name, (region2d, mdr_cells, N, cases) in maps.items():
        d = gen(G, CA, R, np.asarray(region2d, float), np.asarray(mdr_cells), N, cases, rng)
        for k, v in d.items():
            flat[f"{name}/{k}"] = v
        print(name, cases, "nonzero Resp", int((d["resp"] != 0).sum()), "FeAL<1", int((d["feal"] < 1).sum()))
    np.savez_compressed(os.path.join(HERE, "fear_matrix.npz"), **flat)


if __name__ == "__main__":
    main()
