"""Replay a golden CustomMAEnv trajectory (tests/golden/traj_*.npz) through an implementation
and compare every output with the reference's.

An implementation is a ``stepper`` with
  reset(spawn[N]) -> (obs f32 [K, HW], mask u16 [K])
  step(rl[K], scripted[N-K], spawn_next[N] | None) -> dict with keys
     act, mdr, final_pos, crash_bits, restr_bits, reward, fear, shaped, term, trunc,
     crashes, apples, done, ep_return, ep_fear, ep_len, obs, final_obs, mask
Positions, collisions, dones, obs, masks and integer rewards must be bit-exact; FeAR and the
shaped/returned f64 values must be bit-exact too (the tolerance of north_star, 1e-6, is the
documented bound, but the restatement reproduces numpy's operation order exactly).
"""
import numpy as np

FLOAT_TOL = 1e-6  # north_star tolerance for rewards; we assert exact and report the max error


def load(path, seed):
    z = np.load(path)
    d = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(f"s{seed}/")}
    meta = {k: z[k] for k in ("W", "N", "K", "fear", "fear_weight")}
    return d, meta


def replay(stepper, d, K, N, max_err=None):
    reset_at = list(d["reset_at"])
    reset_pos = d["reset_pos"]
    obs, mask = stepper.reset(reset_pos[0])
    np.testing.assert_array_equal(np.round(np.asarray(obs).reshape(d["reset_obs"][0].shape) * 2).astype(np.int8), d["reset_obs"][0], err_msg="reset obs")
    np.testing.assert_array_equal(mask, d["reset_mask"][0], err_msg="reset mask")
    T = len(d["rl"])
    nres = 1
    errs = []
    for t in range(T):
        spawn_next = None
        if d["done"][t]:
            assert reset_at[nres] == t
            spawn_next = reset_pos[nres]
        o = stepper.step(d["rl"][t], d["act"][t][K:], spawn_next)
        ctx = f"step {t}"
        np.testing.assert_array_equal(o["act"], d["act"][t], err_msg=ctx + " actions")
        np.testing.assert_array_equal(o["mdr"], d["mdr"][t], err_msg=ctx + " mdr")
        np.testing.assert_array_equal(o["final_pos"], d["pos"][t], err_msg=ctx + " positions")
        assert int(o["crash_bits"]) == int(d["crash_bits"][t]), ctx + " crash bits"
        assert int(o["restr_bits"]) == int(d["restr_bits"][t]), ctx + " restricted bits"
        np.testing.assert_array_equal(o["reward"], d["reward"][t], err_msg=ctx + " reward")
        np.testing.assert_array_equal(o["fear"], d["fear"][t], err_msg=ctx + " fear")
        np.testing.assert_array_equal(o["shaped"], d["shaped"][t], err_msg=ctx + " shaped")
        errs.append(np.max(np.abs(np.asarray(o["shaped"]) - d["shaped"][t])))
        np.testing.assert_array_equal(o["term"], d["term"][t], err_msg=ctx + " term")
        np.testing.assert_array_equal(o["trunc"], d["trunc"][t], err_msg=ctx + " trunc")
        assert int(o["crashes"]) == int(d["crashes"][t]), ctx + " crashes"
        assert int(o["apples"]) == int(d["apples"][t]), ctx + " apples"
        assert int(o["done"]) == int(d["done"][t]), ctx + " done"
        assert o["ep_return"] == d["ep_return"][t], ctx + " ep_return"
        assert o["ep_fear"] == d["ep_fear"][t], ctx + " ep_fear"
        assert int(o["ep_len"]) == int(d["ep_len"][t]), ctx + " ep_len"
        if d["done"][t]:
            np.testing.assert_array_equal(np.round(np.asarray(o["final_obs"]).reshape(d["obs"][t].shape) * 2).astype(np.int8), d["obs"][t], err_msg=ctx + " final obs")
            np.testing.assert_array_equal(np.round(np.asarray(o["obs"]).reshape(d["obs"][t].shape) * 2).astype(np.int8), d["reset_obs"][nres], err_msg=ctx + " reset obs")
            np.testing.assert_array_equal(o["mask"], d["reset_mask"][nres], err_msg=ctx + " reset mask")
            nres += 1
        else:
            np.testing.assert_array_equal(np.round(np.asarray(o["obs"]).reshape(d["obs"][t].shape) * 2).astype(np.int8), d["obs"][t], err_msg=ctx + " obs")
            np.testing.assert_array_equal(o["mask"], d["mask"][t], err_msg=ctx + " mask")
    return T, (max(errs) if errs else 0.0)


SINGLE = "single_traj.npz"


def single_cases(gold_dir):
    """Run tags of tests/golden/single_traj.npz (make_golden_single.py)."""
    import os
    z = np.load(os.path.join(gold_dir, SINGLE))
    return sorted({k.split("/", 1)[0] for k in z.files})


def load_single(gold_dir, tag):
    import os
    z = np.load(os.path.join(gold_dir, SINGLE))
    return {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(tag + "/")}


def replay_single(stepper, d):
    """Replay a single-agent CustomEnv trajectory (custom/customenv.py:78-183, K = 1) with a
    stepper built for variant 1 and fear_weight 0 (so ep_return is the env's episode reward)."""
    reset_at, reset_pos = list(d["reset_at"]), d["reset_pos"]
    obs, _ = stepper.reset(reset_pos[0])
    shape = d["reset_obs"][0].shape
    q = lambda o: np.round(np.asarray(o).reshape(shape) * 2).astype(np.int8)
    np.testing.assert_array_equal(q(obs), d["reset_obs"][0], err_msg="reset obs")
    nres = 1
    T = len(d["rl"])
    for t in range(T):
        spawn_next = reset_pos[nres] if d["done"][t] else None
        if d["done"][t]:
            assert reset_at[nres] == t
        o = stepper.step([d["rl"][t]], d["act"][t][1:], spawn_next)
        ctx = f"step {t}"
        np.testing.assert_array_equal(o["act"], d["act"][t], err_msg=ctx + " actions")
        np.testing.assert_array_equal(o["mdr"], d["mdr"][t], err_msg=ctx + " mdr")
        np.testing.assert_array_equal(o["final_pos"], d["pos"][t], err_msg=ctx + " positions")
        assert int(o["crash_bits"]) == int(d["crash_bits"][t]), ctx + " crash bits"
        assert (int(o["restr_bits"]) & 1) == int(d["restricted"][t]), ctx + " info['restricted']"
        assert float(o["reward"][0]) == float(d["reward"][t]), (ctx + " reward", o["reward"][0], d["reward"][t])
        assert float(o["fear"][0]) == float(d["fear"][t]), ctx + " info['fear']"
        assert int(o["term"][0]) == int(d["term"][t]), ctx + " terminated"
        assert int(o["trunc"][0]) == int(d["trunc"][t]), ctx + " truncated"
        assert int(o["done"]) == int(d["done"][t]), ctx + " done"
        assert float(o["ep_return"]) == float(d["ep_r"][t]), ctx + " info['episode']['r']"
        assert int(o["ep_len"]) == int(d["ep_l"][t]), ctx + " info['episode']['l']"
        if d["done"][t]:
            np.testing.assert_array_equal(q(o["final_obs"]), d["obs"][t], err_msg=ctx + " final obs")
            np.testing.assert_array_equal(q(o["obs"]), d["reset_obs"][nres], err_msg=ctx + " reset obs")
            nres += 1
        else:
            np.testing.assert_array_equal(q(o["obs"]), d["obs"][t], err_msg=ctx + " obs")
    return T
