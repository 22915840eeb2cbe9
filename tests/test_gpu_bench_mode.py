"""The exact configuration bench.py times, pinned to the C oracle.

bench.py (default, C3) runs VecGridEnv("grid32", 65536 envs, FeAR on, weight -5, max_steps 150,
seed 42, env_offset 0, stats on) with async obs writes (gw_set_obs_async(True): the obs writer of
step t overlaps the world update + FeAR of step t+1) on the default ``defer`` kernel path, and no
host synchronisation inside the stepping loop.  This test steps that env for 170 steps the same
way (every step's obs goes to one of 8 ring buffers, fenced only every 4 steps, so the
descriptor double-buffering is exercised as in the bench) and compares, bit for bit, every output
of a contiguous slice of envs that straddles step_v2 / fear_v2 / obs_kernel block boundaries AND
of envs whose first episode ran into the 150-step cap (maddpg/agent.py:243-247), including the
auto-reset observation after the cap.  Size-independent properties cover all 65,536 envs.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu

E, T, MAX_STEPS, SEED, WEIGHT = 65536, 170, 150, 42, -5.0
SLICE0, SLICE = 4096 - 128, 256          # straddles env 4096 (block edges of every kernel)
PER_STEP = ("reward", "fear", "shaped", "term", "trunc", "done", "mask", "crashes", "apples", "ep_return",
            "ep_fear", "ep_len")


def _bench_env():
    env = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=WEIGHT, max_steps=MAX_STEPS, auto_reset=True,
                     seed=SEED, env_offset=0, stats=True)
    env.set_obs_async(True)  # bench.py: obs_mode True for C3 (537 MB of obs per step >= 128 MB)
    return env


@pytest.fixture(scope="module")
def bench_run(request):
    mp = pytest.MonkeyPatch()
    mp.delenv("GW_KERNEL", raising=False)  # the default path (defer) as in bench.py
    try:
        # pass 1: which envs hit the cap (first episode cut at step 150)
        env = _bench_env()
        env.reset()
        capped_at = torch.full((E,), -1, dtype=torch.int32, device=env.device)
        for t in range(T):
            r = env.step()
            hit = (r.done != 0) & (r.ep_len == MAX_STEPS) & (capped_at < 0)
            capped_at = torch.where(hit, torch.full_like(capped_at, t), capped_at)
        env.obs_fence()
        torch.cuda.synchronize()
        env.close()
        capped_at = capped_at.cpu().numpy()
        capped = np.nonzero(capped_at >= 0)[0]
        cand = [(int(g), int(capped_at[g])) for g in capped if not SLICE0 <= g < SLICE0 + SLICE]
        # 12 envs whose FIRST episode hit the cap, 12 whose capped episode followed shorter ones
        pick = [c for c in cand if c[1] == MAX_STEPS - 1][:12] + [c for c in cand if c[1] > MAX_STEPS - 1][:12]
        sel = np.concatenate([np.arange(SLICE0, SLICE0 + SLICE), np.array([g for g, _ in pick], np.int64)])

        # pass 2: the bench's stepping with per-step captures of the selected envs
        env = _bench_env()
        dev = env.device
        idx = torch.as_tensor(sel, device=dev)
        ring = torch.empty((8, env.K, E, env.H, env.W), dtype=torch.float32, device=dev)
        obs0, mask0 = env.reset()
        env.obs_fence()
        got = {n: [] for n in PER_STEP + ("pos", "obs")}
        reset_obs = obs0[:, idx].clone()
        full = dict(bad_stats=torch.zeros((), dtype=torch.int64, device=dev),
                    capped=torch.zeros((), dtype=torch.int64, device=dev))
        for t in range(T):
            r = env.step(obs_out=ring[t % 8])
            for n in PER_STEP:  # stream-ordered without a fence (sync outputs of the defer path)
                got[n].append(getattr(r, n)[idx].clone())
            got["pos"].append(env.state()["pos"][:, idx].clone())
            st = r.stats.sum(0)
            d = r.done != 0
            # size-independent properties over all 65,536 envs, on the device
            full["bad_stats"] += (st[7] != E).long() + (st[1] != d.sum()).long()
            full["bad_stats"] += (st[6] != r.ep_len[d].sum()).long() + (st[3] != r.crashes.sum()).long()
            full["bad_stats"] += ((st[0] - r.ep_return[d].sum()).abs() > 1e-6 * (1 + r.ep_return[d].abs().sum())).long()
            full["capped"] += ((r.ep_len == MAX_STEPS) & d).sum()
            if t % 4 == 3 or t == T - 1:  # fence every 4 steps: the writer runs ahead meanwhile
                env.obs_fence()
                for u in range(t - (t % 4), t + 1):
                    got["obs"].append(ring[u % 8][:, idx].clone())
        env.obs_fence()
        torch.cuda.synchronize()
        env.close()
        host = {n: torch.stack(v).cpu().numpy() for n, v in got.items()}
        host["reset_obs"] = reset_obs.cpu().numpy()
        full = {k: int(v) for k, v in full.items()}
        return sel, pick, host, full
    finally:
        mp.undo()


def _oracle_run(sc, offset, count):
    """The oracle's outputs for global envs [offset, offset + count) over T steps."""
    orc = O.OracleEnvs(sc, count, fear=True, fear_weight=WEIGHT, max_steps=MAX_STEPS, seed=SEED, env_offset=offset,
                       reset=False)
    obs = np.zeros((sc.K, count, sc.HW), np.float32)
    orc.reset_all(obs=obs, nthreads=16)
    res = {n: [] for n in PER_STEP + ("pos", "obs")}
    res["reset_obs"] = obs.copy()
    outs = (O.StepOut * count)()
    K, N = sc.K, sc.N
    for _ in range(T):
        orc.vec_step(None, obs=obs, outs=outs, nthreads=16)
        o = [outs[e] for e in range(count)]
        res["reward"].append([list(x.reward)[:K] for x in o])
        res["fear"].append([list(x.fear)[:K] for x in o])
        res["shaped"].append([list(x.shaped)[:K] for x in o])
        res["term"].append([list(x.term)[:K] for x in o])
        res["trunc"].append([list(x.trunc)[:K] for x in o])
        res["mask"].append([list(x.mask)[:K] for x in o])
        for n, f in (("done", "done"), ("crashes", "crashes"), ("apples", "apples_caught"), ("ep_return", "ep_return"),
                     ("ep_fear", "ep_fear"), ("ep_len", "ep_len")):
            res[n].append([getattr(x, f) for x in o])
        res["pos"].append(orc.positions().T.copy())
        res["obs"].append(obs.copy())
    return {n: np.asarray(v) for n, v in res.items()}


def _check(host, cols, ref, what):
    for n in PER_STEP:
        g = host[n][:, cols]
        if n == "mask":
            g = g.astype(np.uint16)
        np.testing.assert_array_equal(g, np.asarray(ref[n]).astype(g.dtype), err_msg=f"{what}: {n}")
    np.testing.assert_array_equal(host["pos"][:, :, cols], ref["pos"], err_msg=f"{what}: positions")
    np.testing.assert_array_equal(host["reset_obs"][:, cols].reshape(ref["reset_obs"].shape), ref["reset_obs"],
                                  err_msg=f"{what}: reset obs")
    g = host["obs"][:, :, cols].reshape(ref["obs"].shape)
    for t in range(T):
        np.testing.assert_array_equal(g[t], ref["obs"][t], err_msg=f"{what}: obs at step {t}")


def test_bench_mode_slice_matches_oracle(bench_run):
    sel, pick, host, full = bench_run
    sc = S.builtin("grid32")
    ref = _oracle_run(sc, SLICE0, SLICE)
    _check(host, np.arange(SLICE), ref, f"envs [{SLICE0}, {SLICE0 + SLICE})")
    assert full["bad_stats"] == 0, "per-block statistics disagree with the per-env outputs"
    assert int(np.asarray(ref["done"]).sum()) > 0


def test_bench_mode_capped_episodes_match_oracle(bench_run):
    """Envs with an episode cut at the 150-step cap (the first such episode ends at step index
    ``t_cap``, after 0+ shorter episodes): done / ep_len / ep_return at the cap and the auto-reset
    episode after it, bit-exact."""
    sel, pick, host, full = bench_run
    assert len(pick) > 0 and full["capped"] > 0, "no episode reached the cap"
    sc = S.builtin("grid32")
    assert any(t_cap == MAX_STEPS - 1 for _, t_cap in pick) and any(t_cap > MAX_STEPS - 1 for _, t_cap in pick)
    for j, (g, t_cap) in enumerate(pick):
        ref = _oracle_run(sc, g, 1)
        col = np.array([SLICE + j])
        assert MAX_STEPS - 1 <= t_cap < T
        assert int(np.asarray(ref["ep_len"])[t_cap, 0]) == MAX_STEPS and ref["done"][t_cap][0]
        _check(host, col, ref, f"capped env {g}")
