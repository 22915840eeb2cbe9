"""ReplayRing semantics (a15): what ``sample`` returns == what the reference's per-step loop
stores with ``memory.save_to_memory(state, cont_actions, reward, next_state, termination)``
(maddpg/agent.py:190-197; agilerl MultiAgentReplayBuffer, uniform sampling).

A plain, second env with the same seed is stepped with the actions the rollout chose, and a
per-step copy buffer keeps (state = obs_t, probs_t, shaped reward_t, next_state = the terminal obs
for envs that ended at t else obs_{t+1}, termination_t).  The zero-copy ring (the env writes
obs_{t+1} into slot t+1, terminal obs into a parallel ring, probs written by the fused actor) must
hand out exactly those entries for every sampled (step, env).
"""
import pytest
import torch

from marlnav import scenario as S
from marlnav.actor import MultiAgentActors
from marlnav.rollout import Rollout
from marlnav.vec_env import VecGridEnv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("obs_async,fear_async,slots", [(False, False, 5), (True, False, 5), ("lazy", False, 7),
                                                         ("lazy", True, 4)])
def test_ring_sample_equals_per_step_copy(obs_async, fear_async, slots):
    sc = S.builtin("grid32")
    E, T = 384, 23
    mk = lambda **kw: VecGridEnv(sc, num_envs=E, fear=True, fear_weight=-5.0, max_steps=12, seed=8, stats=True, **kw)
    env, plain = mk(), mk(final_obs=True)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device=env.device, seed=4)
    ro = Rollout(env, actors, replay_slots=slots, training=True, seed=6, obs_async=obs_async, fear_async=fear_async)
    assert ro.fused
    ro.reset()
    obs_p, _ = plain.reset()
    copy = []  # per step: (state, probs, reward, next_state, term)
    for t in range(T):
        state = obs_p.clone()
        ro.step()
        acts = ro._actions.clone()
        probs = ro.replay.probs[t % ro.replay.S].clone()
        r = plain.step(acts)
        done = (r.done != 0)[None, :, None, None]
        nxt = torch.where(done, r.final_obs, r.obs).clone()
        copy.append((state, probs, r.shaped.clone(), nxt, r.term.clone()))
        obs_p = r.obs
    ro.fence()
    rp = ro.replay
    assert int(rp.t_dev) == rp.t == T
    g = torch.Generator(device=env.device).manual_seed(1)
    state, probs, rew, nxt, term, (slot, envi) = rp.sample(4096, generator=g, return_idx=True)
    slot, envi = slot.cpu(), envi.cpu()
    n_win = min(T, rp.S - 1)
    steps = T - 1 - ((T - 1 - slot) % rp.S)        # the step whose transition lives in that slot
    assert int(steps.min()) >= T - n_win and int(steps.max()) == T - 1
    assert len(set(steps.tolist())) == n_win        # every transition of the window is reachable
    dones = 0
    for i in range(4096):
        t, e = int(steps[i]), int(envi[i])
        cs, cp, cr, cn, ct = copy[t]
        assert torch.equal(state[:, i], cs[:, e]), (i, t, e, "state")
        assert torch.equal(probs[:, i], cp[:, e]), (i, t, e, "probs")
        assert torch.equal(rew[i], cr[e]), (i, t, e, "reward")
        assert torch.equal(nxt[:, i], cn[:, e]), (i, t, e, "next_state")
        assert torch.equal(term[i], ct[e]), (i, t, e, "term")
        dones += int(rp.done[int(slot[i]), e])
    assert dones > 0  # terminal transitions (next_state = final obs) were sampled
    env.close()
    plain.close()


def test_reset_mid_rollout_keeps_ring_count():
    """Rollout.reset() with the FeAR-async pipeline: the pending tick is reduced before the ring's
    step count restarts, so after fence() t_dev == the host count."""
    sc = S.builtin("grid32")
    env = VecGridEnv(sc, num_envs=256, fear=True, fear_weight=-5.0, seed=2, stats=True)
    actors = MultiAgentActors(sc.K, sc.H, sc.W, "mlp", device=env.device, seed=1)
    ro = Rollout(env, actors, replay_slots=4, training=True, obs_async="lazy", fear_async=True)
    ro.reset()
    for _ in range(3):
        ro.step()
    ro.reset()
    for _ in range(2):
        ro.step()
    ro.fence()
    assert int(ro.replay.t_dev) == ro.replay.t == 2
    assert ro.totals()["env_steps"] == 5 * 256
    env.close()
