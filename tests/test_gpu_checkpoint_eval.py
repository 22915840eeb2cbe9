"""The reference's trained agents (tests/golden/ckpt_actors.npz: the actor weights of
models/custom/single/level3/{fear/Single_MADDPG_4k, wo_fear/Single_MADDPG}.pt, read without
unpickling by marlnav/checkpoint.py; tests/golden/make_golden_checkpoint.py) on the HIP path.

* The fused actor (gw_actor_act) with those weights, on the single-agent env (variant 1) replaying
  the reference's own trajectories (tests/golden/single_traj.npz: spawns and every agent's
  actions injected, so the env's observation IS the reference's at every step): its logits ==
  the PyTorch fp32 forward of the same weights on the recorded reference obs, within the fused
  actor's stated f32 tolerance (tests/test_actor_ops.py: 2e-4), and its eval-mode action ==
  the masked argmax of those logits outside near-ties.
* ``customeval`` of the trained policy (marlnav/evaluate.py, eval mode, 128 episodes, TRAIN_STEPS
  150, fear off as customeval.py runs it): crashes / apples / steps == the C oracle fed the same
  actions.  The totals are printed (they are the trained agent's, not a parity target: agilerl's
  own get_action is absent, parity unpinned there).
"""
import os

import numpy as np
import pytest
import torch

from marlnav import checkpoint as ck
from marlnav import scenario as S
from marlnav.vec_env import VecGridEnv
from oracle import oracle as O

from _replay import load_single, single_cases

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TAGS = ["level3_fear_4k", "level3_wofear"]


def _actors(tag):
    z = np.load(os.path.join(GOLD, "ckpt_actors.npz"))
    return ck.load_actors([ck.actor_state(z, tag=tag)], 10, 16, device="cuda")


@pytest.mark.parametrize("tag", TAGS)
def test_fused_actor_on_reference_trajectories(tag):
    actors = _actors(tag)
    sc = S.builtin("level3_single")
    logits = torch.empty((1, 1, 9), dtype=torch.float32, device="cuda")
    n_cmp = n_tie = 0
    for case in single_cases(GOLD):
        d = load_single(GOLD, case)
        env = VecGridEnv(sc, num_envs=1, fear=case.startswith("fear"), fear_weight=0.0, max_steps=150,
                         auto_reset=True, final_obs=True, debug=True, variant=1)
        reset_pos = d["reset_pos"]
        env.reset(spawn=torch.as_tensor(reset_pos[0].astype(np.int32)).view(1, -1))
        cur = d["reset_obs"][0]
        nres = 1
        all_obs, fused, acts, masks = [], [], [], []
        for t in range(len(d["rl"]) + 1):
            a, _ = actors.act_env(env, env.out["mask"], training=False, logits_out=logits)
            all_obs.append(cur)
            fused.append(logits[0, 0].clone())
            acts.append(a[0, 0].clone())
            masks.append(env.out["mask"][0, 0].clone())
            if t == len(d["rl"]):
                break
            sp = None
            if d["done"][t]:
                sp = reset_pos[nres].astype(np.int32).reshape(1, -1)
            env.step(np.asarray([[d["rl"][t]]], np.int32), d["act"][t][1:].astype(np.int32).reshape(1, -1), sp)
            if d["done"][t]:
                cur = d["reset_obs"][nres]
                nres += 1
            else:
                cur = d["obs"][t]
        env.close()
        obs = torch.from_numpy(np.stack(all_obs).astype(np.float32) / 2).to("cuda")  # int8 half-units
        with torch.no_grad():
            want = actors(obs.reshape(1, -1, 10, 16))[0]
        got = torch.stack(fused)
        torch.testing.assert_close(got, want, rtol=2e-4, atol=2e-4)
        # eval-mode action = first maximum of the masked softmax (ma_customenv action mask), i.e.
        # of the masked logits; compared where the top two allowed logits are further apart than
        # the logit tolerance (a trained policy's softmax saturates, so probabilities cannot tell)
        bits = (torch.stack(masks).to(torch.int32).unsqueeze(-1) >> torch.arange(9, device="cuda")) & 1
        lm = torch.where(bits.bool(), want, torch.full((), float("-inf"), device="cuda"))
        top2 = lm.topk(2, -1).values
        clear = (top2[:, 0] - top2[:, 1]) > 1e-3
        torch.testing.assert_close(torch.stack(acts)[clear].long(), lm.argmax(-1)[clear])
        n_cmp += int(clear.sum())
        n_tie += int((~clear).sum())
    print(f"{tag}: {n_cmp} actions compared, {n_tie} near-ties skipped")
    assert n_cmp > 2500


@pytest.mark.parametrize("tag", TAGS)
def test_trained_policy_customeval_matches_oracle(tag):
    from marlnav.evaluate import evaluate
    actors = _actors(tag)
    sc = S.builtin("level3_single")
    E, T = 128, 150
    r = evaluate(actors, sc, episodes=E, max_steps=T, fear=False, seed=42, record_actions=True, variant=1)
    acts = r["actions"].cpu().numpy()
    orc = O.OracleEnvs(sc, E, fear=False, fear_weight=0.0, max_steps=T, seed=42, reset=False, variant=1)
    obs_o = np.zeros((sc.K, E, sc.HW), np.float32)
    orc.reset_all(obs=obs_o)
    outs = (O.StepOut * E)()
    active = np.ones(E, bool)
    crashes = apples = steps = 0
    for t in range(acts.shape[0]):
        orc.vec_step(acts[t], obs=obs_o, outs=outs, nthreads=8, auto_reset=False)
        for e in range(E):
            if active[e]:
                crashes += outs[e].crashes
                apples += outs[e].apples_caught
                steps += 1
        active &= ~np.array([bool(outs[e].done) for e in range(E)])
    assert (r["crashes"], r["apples_caught"], r["steps"]) == (crashes, apples, steps)
    print(f"{tag}: {E} episodes: destinations reached {r['apples_caught']}, crashes {r['crashes']}, "
          f"steps {r['steps']}")
