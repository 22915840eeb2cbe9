"""Pin the C restatement (oracle/) against the golden vectors taken from the reference Python.

CPU only.  If these pass, the oracle reproduces custom/grid_world.py, custom/Responsibility.py,
custom/ma_customenv.py and the rollout arithmetic of maddpg/agent.py bit-for-bit on every
recorded input, and can be trusted as the checker of the HIP path.
"""
import glob
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from marlnav import scenario as S

from _replay import load, load_single, replay, replay_single, single_cases

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    assert list(O.philox([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(O.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_np_sum_matches_numpy():
    rng = np.random.default_rng(0)
    for n in [1, 2, 4, 7, 8, 9, 15, 16, 17, 31, 64, 100, 128, 129, 300]:
        for _ in range(50):
            a = rng.standard_normal(n) * 10.0 ** rng.uniform(-4, 4, n)
            assert O.np_sum(a) == np.sum(a)
    for N in (3, 4, 5, 8):
        for _ in range(200):
            R = np.zeros((N, N))
            i = rng.integers(N)
            R[i] = np.clip(rng.integers(-9, 10, N) / (rng.integers(0, 10, N) + 1e-6), -1, 1)
            assert O.np_sum(R) == np.sum(R)


def test_level3_maps_match_reference():
    z = np.load(os.path.join(GOLD, "maps.npz"))
    sc = S.compile_scenario(S.level3_like(10, 16, 4, 2))
    np.testing.assert_array_equal(sc.region.reshape(10, 16), z["region"].astype(np.uint8))
    np.testing.assert_array_equal(sc.policy_map(), z["policy_map"])
    np.testing.assert_array_equal(sc.mdr_map_actions(), z["mdr_action"])
    keys = list(z["policy_keys"])
    assert keys == sc.policy_keys
    np.testing.assert_array_equal(sc.policy_p, z["policy_p"])
    assert [tuple(sc.rc(a)) for a in sc.apples] == [tuple(x) for x in z["apples"]]
    # masks of the table vs the reference's get_action_mask
    for r in range(10):
        for c in range(16):
            assert sc.action_mask[r * 16 + c] == O.lib().orc_action_mask(10, 16, O._ptr(np.ascontiguousarray(sc.region)), r * 16 + c)


def _transition_groups():
    z = np.load(os.path.join(GOLD, "transition.npz"))
    return sorted({k.split("/")[0] for k in z.files if "/" in k})


@pytest.mark.parametrize("group", _transition_groups())
def test_update_world_kats(group):
    z = np.load(os.path.join(GOLD, "transition.npz"))
    g = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(group + "/")}
    H, W = g["region"].shape
    n = len(g["loc"])
    collided = 0
    for i in range(n):
        crash, restr, fin, caught, _ = O.update_world(H, W, g["region"], g["loc"][i], g["act"][i], g["apples"][i])
        np.testing.assert_array_equal(crash, g["crash"][i].astype(bool), err_msg=f"{group} case {i} crash")
        np.testing.assert_array_equal(restr, g["restricted"][i].astype(bool), err_msg=f"{group} case {i} restricted")
        np.testing.assert_array_equal(fin, g["final"][i], err_msg=f"{group} case {i} final")
        exp = [tuple(x) for x in g["caught"][i][: g["n_caught"][i]]]
        assert caught == exp, f"{group} case {i} caught"
        collided += int(crash.any())
    assert collided > 0 or g["loc"].shape[1] == 1


def test_update_world_crafted():
    z = np.load(os.path.join(GOLD, "transition.npz"))
    cases = json.loads(str(z["crafted_json"]))
    region = np.ones(40, np.uint8)
    for c in cases:
        crash, restr, fin, _, _ = O.update_world(5, 8, region, c["loc"], c["act"])
        assert list(crash.astype(int)) == c["crash"]
        assert list(restr.astype(int)) == c["restricted"]
        assert list(fin) == c["final"]


def _fear_groups():
    z = np.load(os.path.join(GOLD, "fear.npz"))
    return sorted({k.split("/")[0] for k in z.files if "/" in k})


@pytest.mark.parametrize("group", _fear_groups())
def test_fear_kats(group):
    z = np.load(os.path.join(GOLD, "fear.npz"))
    g = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(group + "/")}
    H, W = g["region"].shape
    nonzero = 0
    for i in range(len(g["loc"])):
        ids = np.flatnonzero(g["in_list"][i]).astype(np.int32)
        s, resp, vm, va = O.fear_one_actor(H, W, g["region"], g["loc"][i], ids, g["act"][i][ids],
                                           g["mdr"][i], g["actor"][i])
        a = g["actor"][i]
        np.testing.assert_array_equal(vm, g["vm"][i][a], err_msg=f"{group} {i} vm")
        np.testing.assert_array_equal(va, g["va"][i][a], err_msg=f"{group} {i} va")
        np.testing.assert_array_equal(resp, g["resp"][i], err_msg=f"{group} {i} resp")
        assert s == g["sum"][i], f"{group} {i} sum"
        nonzero += int(s != 0)
    assert nonzero > 0


class OracleStepper:
    def __init__(self, sc, fear, weight, variant=0):
        self.o = O.OracleEnvs(sc, 1, fear=fear, fear_weight=weight, max_steps=150, reset=False, variant=variant)
        self.K = sc.K

    def reset(self, spawn):
        return self.o.reset_one(0, spawn=spawn, episode=0)

    def step(self, rl, scripted, spawn_next):
        obs, fobs, out = self.o.step_one(0, rl_act=rl, scripted=scripted, spawn=spawn_next, auto_reset=True)
        K, N = self.K, self.o.sc.N
        return dict(act=list(out.actions)[:N], mdr=list(out.mdr)[:N], final_pos=list(out.final_pos)[:N],
                    crash_bits=out.crash_bits, restr_bits=out.restricted_bits,
                    reward=list(out.reward)[:K], fear=list(out.fear)[:K], shaped=list(out.shaped)[:K],
                    term=list(out.term)[:K], trunc=list(out.trunc)[:K], crashes=out.crashes,
                    apples=out.apples_caught, done=out.done, ep_return=out.ep_return,
                    ep_fear=out.ep_fear, ep_len=out.ep_len, obs=obs, final_obs=fobs,
                    mask=list(out.mask)[:K])


SCEN_OF = {"level3": "level3", "level3like": "level3", "grid32": "grid32", "grid64n8": "grid64_n8"}


def traj_cases():
    cases = []
    for path in sorted(glob.glob(os.path.join(GOLD, "traj_*.npz"))):
        z = np.load(path)
        for s in z["seeds"]:
            cases.append((os.path.basename(path), int(s)))
    return cases


def scenario_for(fname):
    key = fname[len("traj_"):].rsplit("_", 1)[0]
    return S.builtin(SCEN_OF[key])


@pytest.mark.parametrize("fname,seed", traj_cases())
def test_oracle_replays_reference_trajectory(fname, seed):
    d, meta = load(os.path.join(GOLD, fname), seed)
    sc = scenario_for(fname)
    assert sc.N == int(meta["N"]) and sc.K == int(meta["K"])
    st = OracleStepper(sc, bool(meta["fear"]), float(meta["fear_weight"]))
    T, err = replay(st, d, sc.K, sc.N)
    assert T > 0 and err == 0.0


@pytest.mark.parametrize("tag", single_cases(GOLD))
def test_oracle_replays_single_agent_trajectory(tag):
    """custom/customenv.py (single-agent CustomEnv) trajectories from the reference, bit-exact."""
    d = load_single(GOLD, tag)
    st = OracleStepper(S.builtin("level3_single"), tag.startswith("fear"), 0.0, variant=1)
    assert replay_single(st, d) == len(d["rl"])


def _fm_cases():
    z = np.load(os.path.join(GOLD, "fear_matrix.npz"))
    return sorted({k.split("/", 1)[0] for k in z.files})


@pytest.mark.parametrize("name", _fm_cases())
def test_oracle_fear_matrix_and_feal_match_reference(name):
    """Responsibility.FeAR (full matrix) and FeAL golden vectors from the reference, bit-exact."""
    z = np.load(os.path.join(GOLD, "fear_matrix.npz"))
    d = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(name + "/")}
    H, W = d["region"].shape
    for i in range(len(d["loc"])):
        o = O.fear_matrix(H, W, d["region"], d["loc"][i], d["act"][i], d["mdr"][i], d["in_list"][i].astype(bool))
        np.testing.assert_array_equal(o["vm"], d["vm"][i], err_msg=f"{name} case {i} vm")
        np.testing.assert_array_equal(o["va"], d["va"][i], err_msg=f"{name} case {i} va")
        np.testing.assert_array_equal(o["resp"], d["resp"][i], err_msg=f"{name} case {i} resp")
        np.testing.assert_array_equal(o["feal_vm"], d["feal_vm"][i], err_msg=f"{name} case {i} feal vm")
        np.testing.assert_array_equal(o["feal_va"], d["feal_va"][i], err_msg=f"{name} case {i} feal va")
        np.testing.assert_array_equal(o["feal"], d["feal"][i], err_msg=f"{name} case {i} feal")
