"""GPU tests of the host-side pieces around the kernels: the CustomMAEnv facade, the actors and
the batched rollout with the zero-copy replay ring."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from marlnav import scenario as S
from marlnav.actor import MultiAgentActors
from marlnav.rollout import Rollout
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


def test_facade_matches_oracle_native_mode():
    """CustomMAEnv (reference dict API, E = 1, no auto-reset, no step cap) == the oracle."""
    from custom.ma_customenv import CustomMAEnv
    sc = S.builtin("level3")
    env = CustomMAEnv(render=False, fear=True, seed=123)
    orc = O.OracleEnvs(sc, 1, fear=True, fear_weight=0.0, max_steps=0, seed=123, reset=False)
    obs, info = env.reset()
    o_obs, o_mask = orc.reset_one(0, episode=0)
    assert set(obs) == {"agent_0", "agent_1"} and info["fear"] == 0.0
    for k in range(2):
        np.testing.assert_array_equal(obs[f"agent_{k}"], o_obs[k].reshape(10, 16).astype(np.float64))
        assert obs[f"agent_{k}"].dtype == np.float64
        m = info[f"agent_{k}"]["action_mask"]
        assert m.dtype == np.int8 and int(np.dot(m, 1 << np.arange(9))) == int(o_mask[k])
    rng = np.random.default_rng(0)
    for t in range(60):
        a = tuple(int(x) for x in rng.integers(0, 9, 2))
        obs, rew, term, trunc, info = env.step(a)
        o_obs, _, out = orc.step_one(0, rl_act=np.array(a, np.int32), auto_reset=False)
        assert rew == {f"agent_{k}": int(out.reward[k]) for k in range(2)}
        assert all(isinstance(v, int) for v in rew.values())
        assert term == {f"agent_{k}": bool(out.term[k]) for k in range(2)}
        assert trunc == {f"agent_{k}": bool(out.trunc[k]) for k in range(2)}
        assert info["fear"] == {f"agent_{k}": out.fear[k] for k in range(2)}
        assert info["agent_crashes"] == out.crashes and info["apples_caught"] == out.apples_caught
        assert [x[1] for x in env.Action4Agents] == list(out.actions)[:4]
        for k in range(2):
            np.testing.assert_array_equal(obs[f"agent_{k}"], o_obs[k].reshape(10, 16))
    assert env.step(()) == ({}, {}, {}, {}, {})
    assert env.action_space.n == 9 and env.num_agents == 2
    assert env.observation_space("agent_0").shape == (10, 16)


def test_stacked_actor_matches_plain_pytorch_fp32():
    """The batched K-agent MLP == K independent nn.Sequential fp32 actors."""
    torch.manual_seed(0)
    K, H, W, E = 2, 32, 32, 512
    actors = MultiAgentActors(K, H, W, "mlp", device="cuda", seed=3)
    x = torch.randint(-1, 6, (K, E, H, W), device="cuda").float()
    got = actors(x)
    net = actors.net
    for k in range(K):
        ref = torch.nn.Sequential(
            torch.nn.Linear(H * W, 128), torch.nn.LayerNorm(128), torch.nn.ReLU(),
            torch.nn.Linear(128, 128), torch.nn.LayerNorm(128), torch.nn.ReLU(),
            torch.nn.Linear(128, 9)).cuda()
        with torch.no_grad():
            for li, lin in enumerate([ref[0], ref[3], ref[6]]):
                lin.weight.copy_(net.weights[li][k].t())
                lin.bias.copy_(net.biases[li][k, 0])
            for li, ln in enumerate([ref[1], ref[4]]):
                ln.weight.copy_(net.ln_w[li][k, 0])
                ln.bias.copy_(net.ln_b[li][k, 0])
            want = ref(x[k].reshape(E, -1))
        torch.testing.assert_close(got[k], want, rtol=1e-4, atol=1e-4)


def test_rollout_with_actor_and_replay_ring():
    sc = S.builtin("grid32")
    E = 2048
    env = VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, stats=True, final_obs=False, debug=True)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device=env.device, seed=1)
    ro = Rollout(env, actors, replay_slots=4, training=True, seed=2)
    ro.reset()
    shaped_sum = 0.0
    for t in range(40):
        mask = env.out["mask"].clone()
        r = ro.step()
        # actions respect the action mask of the obs they were chosen from
        a = r.actions[:, : sc.K].long()
        allowed = (mask.long() >> a) & 1
        assert bool(allowed.all())
        cur = t % ro.replay.S
        assert torch.equal(ro.replay.reward[cur], r.shaped)
        shaped_sum += float(r.shaped.sum())
    tot = ro.totals()
    assert tot["env_steps"] == 40 * E
    assert abs(tot["shaped"] - shaped_sum) < 1e-6 * max(1.0, abs(shaped_sum))
    state, probs, rew, nxt, term = ro.replay.sample(256)
    assert state.shape == (sc.K, 256, sc.H, sc.W) and nxt.shape == state.shape
    assert probs.shape == (sc.K, 256, 9) and rew.shape == (256, sc.K)
    torch.testing.assert_close(probs.sum(-1), torch.ones_like(probs.sum(-1)))
    env.close()


def test_cnn_actor_runs():
    actors = MultiAgentActors(2, 64, 64, "cnn", device="cuda")
    x = torch.zeros((2, 16, 64, 64), device="cuda")
    a, p = actors.act(x, None, training=False)
    assert a.shape == (16, 2) and p.shape == (2, 16, 9)


def test_graph_learn_equals_eager_learn():
    """The HIP-graph replay of one MADDPG update == the eager update on the same batch and noise."""
    from marlnav.maddpg import MADDPG
    K, H, W, B = 2, 32, 32, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    batch = (torch.randint(-1, 6, (K, B, H, W), device="cuda", generator=g).float(),
             torch.softmax(torch.randn((K, B, 9), device="cuda", generator=g), -1),
             torch.randn((B, K), device="cuda", generator=g, dtype=torch.float64),
             torch.randint(-1, 6, (K, B, H, W), device="cuda", generator=g).float(),
             (torch.rand((B, K), device="cuda", generator=g) < 0.1).to(torch.uint8),
             torch.rand((K, B, 9), device="cuda", generator=g), torch.rand((K, B, 9), device="cuda", generator=g))
    a = MADDPG(K, H, W, device="cuda", seed=1, capturable=True)
    b = MADDPG(K, H, W, device="cuda", seed=1, capturable=True)
    for _ in range(2):  # warm-up updates on both (optimizer state exists before capture)
        a.learn(*batch)
        b.learn(*batch)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(graph):
        out = a.learn(*batch)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        graph.replay()
        want = b.learn(*batch)
    torch.cuda.synchronize()
    torch.testing.assert_close(out[0], want[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out[1], want[1], rtol=1e-5, atol=1e-6)
    for x, y in zip(a.state_dict().values(), b.state_dict().values()):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_trainer_with_graph_learns_and_samples_the_live_window():
    from marlnav.maddpg import MADDPG
    from marlnav.train import MADDPGTrainer
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=512, fear=True, fear_weight=-5.0, stats=True, final_obs=True)
    m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=2, capturable=True)
    w0 = m.actors.net.weights[0].detach().clone()
    tr = MADDPGTrainer(env, m, memory_size=4096, updates_per_step=2, graph=True, seed=3)
    tr.reset()
    s = tr.train(24)
    torch.cuda.synchronize()
    assert s["updates"] > 0 and s["env_steps"] == 24 * 512
    a_loss, c_loss = tr.losses[-1]
    assert torch.isfinite(a_loss).all() and torch.isfinite(c_loss).all()
    assert not torch.equal(w0, m.actors.net.weights[0])
    # sampling indices are computed on device from t_dev: always inside the filled window
    rp = tr.rollout.replay
    *_, (slot, envi) = rp.sample(4096, return_idx=True)
    n = min(rp.t, rp.S - 1)
    age = (rp.t - 1 - slot.cpu().numpy()) % rp.S
    assert age.max() < n and envi.max().item() < env.E
    env.close()


def test_evaluate_matches_oracle():
    """customeval totals (crashes, apples, steps, FeAR) over 64 episodes == the C oracle fed the
    same actions with the same early-stop rule."""
    from marlnav.evaluate import evaluate
    sc = S.builtin("level3")
    E, T = 64, 150
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device="cuda", seed=5)
    r = evaluate(actors, sc, episodes=E, max_steps=T, fear=True, seed=11, record_actions=True)
    acts = r["actions"].cpu().numpy()
    orc = O.OracleEnvs(sc, E, fear=True, fear_weight=-5.0, max_steps=T, seed=11, reset=False)
    obs_o = np.zeros((sc.K, E, sc.HW), np.float32)
    orc.reset_all(obs=obs_o)
    outs = (O.StepOut * E)()
    active = np.ones(E, bool)
    crashes = apples = steps = 0
    fear = 0.0
    alive_before_last = True
    for t in range(acts.shape[0]):
        if t == acts.shape[0] - 1:
            alive_before_last = bool(active.any())
        orc.vec_step(acts[t], obs=obs_o, outs=outs, nthreads=8, auto_reset=False)
        for e in range(E):
            if active[e]:
                crashes += outs[e].crashes
                apples += outs[e].apples_caught
                steps += 1
                fear += sum(outs[e].fear[k] for k in range(sc.K))
        active &= ~np.array([bool(outs[e].done) for e in range(E)])
    assert (r["crashes"], r["apples_caught"], r["steps"]) == (crashes, apples, steps)
    assert abs(r["fear"] - fear) < 1e-9
    assert not active.any() or acts.shape[0] == T
    # the recorded actions end at the first step after which every episode had ended (no extra
    # rows from the every-8-steps early-stop check)
    assert alive_before_last


def test_single_agent_facade_matches_oracle():
    """custom/customenv.py surface (CustomEnv, K = 1) == the C oracle's variant 1, native RNG."""
    from custom.customenv import CustomEnv
    sc = S.builtin("level3_single")
    env = CustomEnv(render=False, fear=True, seed=99)
    orc = O.OracleEnvs(sc, 1, fear=True, fear_weight=0.0, max_steps=0, seed=99, reset=False, variant=1)
    rng = np.random.default_rng(3)
    episode = 0
    obs, info = env.reset()
    o_obs, _ = orc.reset_one(0, episode=episode)
    assert info == {} and obs.shape == (10, 16) and obs.dtype == np.float64
    np.testing.assert_array_equal(obs, o_obs[0].reshape(10, 16))
    ep_r, ep_l, seen_bonus = 0.0, 0, False
    for t in range(400):
        a = int(rng.integers(0, 9))
        obs, rew, term, trunc, info = env.step([a])
        o_obs, _, out = orc.step_one(0, rl_act=np.array([a], np.int32), auto_reset=False)
        ep_r += out.reward[0]
        ep_l += 1
        assert rew == [out.reward[0]] and term == [bool(out.term[0])] and trunc == bool(out.trunc[0])
        assert info["fear"] == out.fear[0] and info["restricted"] == bool(out.restricted_bits & 1)
        assert info["episode"] == {"r": ep_r, "l": ep_l}
        np.testing.assert_array_equal(obs, o_obs[0].reshape(10, 16))
        seen_bonus |= abs(rew[0] - round(rew[0])) > 1e-9
        if term[0] or trunc:
            episode += 1
            obs, _ = env.reset()
            o_obs, _ = orc.reset_one(0, episode=episode)
            np.testing.assert_array_equal(obs, o_obs[0].reshape(10, 16))
            ep_r, ep_l = 0.0, 0
    assert episode > 3 and seen_bonus


def test_rollout_tick_reduces_partials_and_counts():
    """gw_rollout_tick (include/rollout_ops.h) == torch row sum (deterministic order, f64)."""
    from marlnav.parallel import StatsReducer
    g = torch.Generator(device="cuda").manual_seed(4)
    red = StatsReducer(8, "cuda")
    ctr = torch.zeros((), dtype=torch.int64, device="cuda")
    want = torch.zeros(8, dtype=torch.float64, device="cuda")
    for rows in (1, 7, 512, 2561):
        p = torch.randn((rows, 8), dtype=torch.float64, device="cuda", generator=g)
        red.push(p, counter=ctr)
        want += p.sum(0)
    torch.testing.assert_close(red.result(), want, rtol=1e-12, atol=1e-12)
    assert int(ctr) == 4
    again = StatsReducer(8, "cuda")
    again.push(p)
    first = again.result().clone()
    again2 = StatsReducer(8, "cuda")
    again2.push(p)
    assert torch.equal(first, again2.result())  # bit-identical run to run


def test_trainer_checkpoint_resume(tmp_path):
    """MADDPGAgent.save_checkpoint / load_checkpoint (maddpg/agent.py:255-281): networks +
    optimizers, the replay memory and the step counter come back; after resume() the last stored
    transition keeps its next state (read through the final-obs slot) and the ring continues with
    the fresh episodes' obs; the resumed trainer samples, learns and steps on."""
    from marlnav.maddpg import MADDPG
    from marlnav.train import MADDPGTrainer
    sc = S.builtin("grid32")

    def make(seed):
        env = VecGridEnv(sc, num_envs=256, fear=True, fear_weight=-5.0, stats=True, final_obs=True, seed=seed)
        m = MADDPG(sc.K, sc.H, sc.W, device=env.device, seed=seed, capturable=False)
        return env, m, MADDPGTrainer(env, m, memory_size=2048, updates_per_step=1, graph=False, seed=seed)

    env, m, tr = make(2)
    tr.reset()
    tr.train(12)
    rp = tr.rollout.replay
    tr.rollout.fence()
    t = rp.t
    prev = (t - 1) % rp.S
    want_next = rp.obs[t % rp.S].clone()
    tr.save_checkpoint(str(tmp_path), "agent.safetensors")
    env2, m2, tr2 = make(5)
    tr2.reset()
    tr2.load_checkpoint(str(tmp_path), "agent.safetensors")
    rp2 = tr2.rollout.replay
    assert rp2.t == t and int(rp2.t_dev) == int(rp.t_dev) and tr2.total_steps == tr.total_steps
    for n in ("probs", "reward", "term"):
        assert torch.equal(getattr(rp2, n), getattr(rp, n))
    assert torch.equal(rp2.final_obs[prev], want_next) and bool((rp2.done[prev] == 1).all())
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)
    assert torch.equal(m.opt_actor.m, m2.opt_actor.m) and int(m.opt_actor.count[0]) == int(m2.opt_actor.count[0])
    # the fused actor's noise counter continues: no replay of the first run's noise
    assert tr2.rollout._calls == tr.rollout._calls == 12
    assert tr2.rollout._noise_base + rp2.t == tr2.rollout._calls
    u0 = tr2.updates
    tr2.train(3)  # the resumed trainer keeps stepping and learning
    torch.cuda.synchronize()
    assert tr2.updates > u0 and torch.isfinite(tr2.losses[-1][0]).all()
    env.close()
    env2.close()
