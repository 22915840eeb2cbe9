"""Native-RNG mode reproduces the reference's random LAWS (not its streams).

The reference draws scripted actions with numpy's global MT19937 (custom/custom_agent.py:31),
the 25 % uniform-direction branch with Python's unseeded `random` (custom/ma_customenv.py:441)
and spawns with a per-env PCG64 (:97, :376).  The build replaces all three by Philox draws
that are identical on the GPU and in the C oracle (bit-exactness: tests/test_gpu_parity.py).
Here the oracle's draws are checked against the reference's distributions (chi-square)."""
import numpy as np
import pytest
from scipy import stats

from oracle import oracle as O
from marlnav import scenario as S


def _chi2_ok(counts, probs, alpha=1e-4):
    counts = np.asarray(counts, float)
    probs = np.asarray(probs, float)
    keep = probs > 0
    assert counts[~keep].sum() == 0, "drew an action of probability 0"
    exp = probs[keep] / probs[keep].sum() * counts.sum()
    return stats.chisquare(counts[keep], exp).pvalue > alpha


def test_scripted_policy_law():
    """Per-cell policy mixture: 0.75 scenario weights + 0.25 uniform-direction weights."""
    sc = S.builtin("level3")
    E = 4096
    o = O.OracleEnvs(sc, E, fear=False, seed=17)
    outs = (O.StepOut * E)()
    counts = {}
    for t in range(12):
        pos = o.positions()
        o.vec_step(np.zeros((E, sc.K), np.int32), outs=outs, nthreads=8, auto_reset=False)
        for e in range(E):
            for n in range(sc.K, sc.N):
                pid = int(sc.policy_id[pos[e][n]])
                counts.setdefault(pid, np.zeros(9))[outs[e].actions[n]] += 1
    for pid, c in counts.items():
        if c.sum() < 200:
            continue
        p = 0.75 * sc.policy_p[pid, 0] + 0.25 * sc.policy_p[pid, 1]
        assert _chi2_ok(c, p), (sc.policy_keys[pid], c, p)


def test_spawn_law_uniform_subsets_sorted():
    sc = S.builtin("level3")
    E = 20000
    o = O.OracleEnvs(sc, E, fear=False, seed=3)
    pos = o.positions()
    assert np.all(np.diff(pos, axis=1) > 0), "spawns are distinct and sorted row-major"
    assert np.isin(pos, sc.free_cells).all()
    # each road cell is included with probability N / F
    inc = np.bincount(np.searchsorted(sc.free_cells, pos.ravel()), minlength=sc.free_cells.size)
    assert _chi2_ok(inc, np.full(sc.free_cells.size, 1.0 / sc.free_cells.size))
    # pairs: P(cell a and cell b both chosen) is the same for every pair (uniform subsets)
    F = sc.free_cells.size
    idx = np.searchsorted(sc.free_cells, pos)
    first_two = np.bincount(idx[:, 0] * F + idx[:, 1], minlength=F * F).reshape(F, F)
    # the sorted minimum follows the law of the minimum of a uniform 4-subset
    mins = np.bincount(idx[:, 0], minlength=F)
    from math import comb
    pmin = np.array([comb(F - 1 - m, sc.N - 1) for m in range(F)], float)
    assert _chi2_ok(mins, pmin / pmin.sum())
    assert first_two.sum() == E


def test_random_rl_policy_uniform():
    sc = S.builtin("grid32")
    E = 8192
    o = O.OracleEnvs(sc, E, fear=False, seed=5)
    outs = (O.StepOut * E)()
    c = np.zeros(9)
    for _ in range(4):
        o.vec_step(None, outs=outs, nthreads=8)
        for e in range(E):
            for k in range(sc.K):
                c[outs[e].actions[k]] += 1
    assert _chi2_ok(c, np.full(9, 1 / 9))


@pytest.mark.parametrize("name", ["level3", "grid32"])
def test_episode_statistics_plausible(name):
    """Random-policy episodes end by crash / apples / cap like the reference's (mean
    length ~12.6 on Level 3 under random RL actions, crash dominated)."""
    sc = S.builtin(name)
    E = 2048
    o = O.OracleEnvs(sc, E, fear=False, seed=11)
    outs = (O.StepOut * E)()
    lens, crashes, apples = [], 0, 0
    for _ in range(200):
        o.vec_step(None, outs=outs, nthreads=8)
        for e in range(E):
            crashes += outs[e].crashes
            apples += outs[e].apples_caught
            if outs[e].done:
                lens.append(outs[e].ep_len)
    lens = np.array(lens)
    assert lens.max() <= 150 and lens.min() >= 1
    assert crashes > apples
    if name == "level3":
        assert 8 < lens.mean() < 20
