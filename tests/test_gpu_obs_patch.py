"""Egocentric local observations (gw_obs_patch, VecGridEnv.obs_patch).

Not a reference feature: the reference observes the whole relabelled grid
(custom/ma_customenv.py:303-322), which stays the parity path.  The patch format is checked
against the full-grid observation it is derived from: agent k's P x P window == the full obs of
agent k, padded with -1 (the inactive-cell value), cropped around k's cell (rows / cols
-P/2 .. P-1-P/2).  The full obs is itself pinned to the oracle (test_gpu_parity.py).  Covered:
odd and even P, windows larger than the grid, agents on the border, auto-reset (the window of
the new episode's spawn), terminal windows of done envs (centred on the terminal cell), async
obs, and an env run without dense obs at all."""
import pytest
import torch
import torch.nn.functional as F

from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def crop(full, centers, P, W):
    """full [E, H, W] obs of one agent, centers [E] cells -> [E, P, P] windows (pad -1)."""
    lo, hi = P // 2, P - 1 - P // 2
    pad = F.pad(full, (lo, hi, lo, hi), value=-1.0)
    r, c = centers // W, centers % W
    dy = torch.arange(P, device=full.device)
    rows = (r[:, None] + dy[None, :])                        # [E, P] rows of the padded grid
    cols = (c[:, None] + dy[None, :])
    e = torch.arange(full.shape[0], device=full.device)
    return pad[e[:, None, None], rows[:, :, None], cols[:, None, :]]


@pytest.mark.parametrize("scen,E,P,fear,async_obs", [("grid32", 2048, 11, True, False), ("grid32", 777, 8, False, True),
                                                     ("level3", 300, 5, True, False), ("level3", 64, 40, False, False),
                                                     ("grid64_n8", 512, 15, True, "lazy"),
                                                     ("grid64_n8", 1000, 16, False, True), ("level3", 50, 4, True, False)])
def test_patch_equals_cropped_full_obs(scen, E, P, fear, async_obs):
    env = VecGridEnv(scen, num_envs=E, fear=fear, fear_weight=-5.0, max_steps=15, seed=7, final_obs=True, debug=True)
    if async_obs:
        env.set_obs_async(async_obs)
    env.reset()
    env.obs_fence()
    K, W = env.K, env.W
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    done_seen = torch.zeros((), dtype=torch.int64, device="cuda")
    pos = env.state()["pos"]                                   # [N, E]
    p = env.obs_patch(P)
    for k in range(K):
        bad += (p[k] != crop(env.out["obs"][k], pos[k], P, W)).sum()
    for t in range(30):
        r = env.step()
        patch, fin = env.obs_patch(P, final=True)
        env.obs_fence()
        pos = env.state()["pos"]
        d = r.done != 0
        done_seen += d.sum()
        for k in range(K):
            bad += (patch[k] != crop(r.obs[k], pos[k], P, W)).sum()
            ref_f = crop(r.final_obs[k], r.final_pos[:, k].contiguous(), P, W)
            bad += (fin[k][d] != ref_f[d]).sum()
            bad += (~torch.isnan(fin[k][~d])).sum()          # terminal windows only for done envs
    torch.cuda.synchronize()
    assert int(done_seen) > 0
    assert int(bad) == 0
    env.close()


@pytest.mark.parametrize("K,P", [(8, 16), (8, 32), (8, 23), (2, 64), (2, 100)])
def test_patch_large_windows_and_many_agents(K, P):
    """The K x P combinations whose LDS exceeds the 64 KB a launch gets by default (before
    cca6a63 they failed to launch; until round 4 they fell back to the per-element writer): with
    all 8 world agents learning (K = 8, 64 x 64) the nibble table of P = 16 (70 KB of LDS) and the
    byte table of P = 32 / odd P = 23 run with the dynamic-LDS attribute raised; P = 64 (141 KB,
    K = 2) too; P = 100 (a 320 KB table) takes the per-element writer.  Every window == the
    -1-padded crop of the full obs, terminal windows included."""
    from marlnav import scenario as S
    sc = S.compile_scenario(S.level3_like(64, 64, 8, K), name=f"grid64_n8_k{K}")
    E = 300
    env = VecGridEnv(sc, num_envs=E, fear=False, max_steps=12, seed=5, final_obs=True, debug=True)
    env.reset()
    W = env.W
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    done_seen = torch.zeros((), dtype=torch.int64, device="cuda")
    pos = env.state()["pos"]
    p = env.obs_patch(P)
    for k in range(K):
        bad += (p[k] != crop(env.out["obs"][k], pos[k], P, W)).sum()
    for t in range(16):
        r = env.step()
        patch, fin = env.obs_patch(P, final=True)
        pos = env.state()["pos"]
        d = r.done != 0
        done_seen += d.sum()
        for k in range(K):
            bad += (patch[k] != crop(r.obs[k], pos[k], P, W)).sum()
            ref_f = crop(r.final_obs[k], r.final_pos[:, k].contiguous(), P, W)
            bad += (fin[k][d] != ref_f[d]).sum()
    torch.cuda.synchronize()
    assert int(done_seen) > 0
    assert int(bad) == 0
    env.close()


def test_patch_without_dense_obs():
    """obs=False: no full-grid obs is written at all, the patches still come from the descriptors."""
    a = VecGridEnv("grid32", num_envs=1000, fear=True, seed=3, max_steps=20)
    b = VecGridEnv("grid32", num_envs=1000, fear=True, seed=3, max_steps=20, obs=False)
    a.reset()
    b.reset()
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(25):
        a.step()
        b.step()
        bad += (a.obs_patch(9) != b.obs_patch(9)).sum()
    torch.cuda.synchronize()
    assert int(bad) == 0
    assert b.out["obs"] is None
    a.close()
    b.close()


def test_patch_rollout_feeds_the_actor_and_the_ring():
    """Rollout(patch=P) on an env without dense obs == a hand loop on a full-obs env that crops
    the windows itself: the same actor inputs (so the same actions / probs with the same
    generator), the same trajectories, and ring slots holding the cropped windows (terminal
    windows of done envs in the final-obs ring)."""
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    E, P, T, S = 1500, 9, 20, 24
    actors = MultiAgentActors(2, P, P, "mlp", device="cuda", seed=4)
    env_p = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=-5.0, seed=11, max_steps=12, obs=False, stats=True)
    ro = Rollout(env_p, actors, replay_slots=S, training=True, seed=6, patch=P, fused=False)  # the torch actor
    assert not ro.fused
    ro.reset()
    env_f = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=-5.0, seed=11, max_steps=12, final_obs=True,
                       debug=True)
    obs, mask = env_f.reset()
    gen = torch.Generator(device="cuda").manual_seed(6)
    W = env_f.W
    pos = env_f.state()["pos"]
    cur = torch.stack([crop(obs[k], pos[k], P, W) for k in range(2)])
    bad = torch.zeros((), dtype=torch.int64, device="cuda")
    done_seen = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(T):
        bad += (ro.replay.obs[t % S] != cur).sum()
        a, probs = actors.act(cur, env_f.out["mask"], True, generator=gen)
        r_p = ro.step()
        bad += (ro.replay.probs[t % S] != probs).sum()
        r = env_f.step(a)
        bad += (r.reward != r_p.reward).sum() + (r.done != r_p.done).sum() + (r.shaped != ro.replay.reward[t % S]).sum()
        d = r.done != 0
        done_seen += d.sum()
        for k in range(2):
            fin = crop(r.final_obs[k], r.final_pos[:, k].contiguous(), P, W)
            bad += (ro.replay.final_obs[t % S][k][d] != fin[d]).sum()
        pos = env_f.state()["pos"]
        cur = torch.stack([crop(r.obs[k], pos[k], P, W) for k in range(2)])
    bad += (ro.replay.obs[T % S] != cur).sum()
    torch.cuda.synchronize()
    assert int(done_seen) > 0
    assert int(bad) == 0
    state, probs, reward, nxt, term = ro.replay.sample(256)
    assert state.shape == (2, 256, P, P) and nxt.shape == (2, 256, P, P)
    env_p.close()
    env_f.close()


@pytest.mark.parametrize("scen,E,P,fear", [("grid32", 4096, 11, True), ("grid64_n8", 2048, 16, True),
                                           ("grid32", 1024, 8, True), ("level3", 64, 4, True),
                                           ("grid32", 1000, 11, False), ("grid32", 1022, 11, True)])
def test_step_patch_next_equals_obs_patch_after_the_step(scen, E, P, fear):
    """gw_step_patch_next + gw_step == gw_step + gw_obs_patch: the windows and terminal windows bit
    for bit, and every step output unchanged, over auto-resets.  FeAR on with E % 4 == 0: the
    windows come from the FeAR launch (fear_rows_kernel); FeAR off or E % 4 != 0: the fallback
    writer after the step."""
    envs = [VecGridEnv(scen, num_envs=E, fear=fear, fear_weight=-5.0, seed=21, max_steps=9, obs=False)
            for _ in range(2)]
    K = envs[0].K
    bufs = [[torch.full((K, E, P, P), float("nan"), device="cuda") for _ in range(2)] for _ in range(2)]
    for env in envs:
        env.reset()
    for t in range(25):
        envs[0].patch_next(P, bufs[0][0], bufs[0][1])
        r0 = envs[0].step()
        r1 = envs[1].step()
        envs[1].obs_patch(P, final=True, out=bufs[1][0], final_out=bufs[1][1])
        assert torch.equal(bufs[0][0], bufs[1][0]), t
        assert torch.equal(torch.nan_to_num(bufs[0][1], nan=7.0), torch.nan_to_num(bufs[1][1], nan=7.0)), t
        for name in ("reward", "done", "shaped", "fear"):
            x, y = getattr(r0, name), getattr(r1, name)
            if x is not None:
                assert torch.equal(x, y), (t, name)
    for env in envs:
        env.close()


@pytest.mark.parametrize("graph", [False, True])
def test_rollout_windows_from_the_fear_launch(graph, monkeypatch):
    """Rollout(patch=P) with the fused MLP window actor and FeAR on writes each step's windows from
    the FeAR launch (default) == the writer after the step (GW_FEAR_PATCH=0): identical ring
    contents, eager and as ring-phase graphs."""
    from marlnav.actor import MultiAgentActors
    from marlnav.rollout import Rollout
    E, P, n = 2048, 11, 4
    actors = MultiAgentActors(2, P, P, "mlp", device="cuda", seed=4)
    rings = []
    for on in ("1", "0"):
        monkeypatch.setenv("GW_FEAR_PATCH", on)
        env = VecGridEnv("grid32", num_envs=E, fear=True, fear_weight=-5.0, seed=13, max_steps=10, obs=False)
        ro = Rollout(env, actors, replay_slots=8, training=True, seed=6, patch=P)
        assert ro.fused
        ro.reset()
        for _ in range(3):
            ro.step()
        if graph:
            g = ro.capture(n)
            for _ in range(3):
                g.replay()
        else:
            for _ in range(3 * n):
                ro.step()
        ro.fence()
        torch.cuda.synchronize()
        rings.append((ro.replay.obs.clone(), ro.replay.probs.clone(), ro.replay.reward.clone(),
                      ro.replay.done.clone(), torch.nan_to_num(ro.replay.final_obs, nan=7.0)))
        env.close()
    for x, y in zip(*rings):
        assert torch.equal(x, y)
