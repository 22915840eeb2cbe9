"""Evaluation driver: ``customeval.py:70-133`` batched.

The reference evaluates a trained MADDPG for ``eval_episodes = 100`` episodes, one env at a
time: every episode runs at most TRAIN_STEPS steps (``configs/custom.yaml``) and stops when all
RL agents are terminated or all are truncated; it sums ``info["agent_crashes"]`` and
``info["apples_caught"]`` over all steps taken and counts the steps.  Here the episodes run as
E = episodes envs in parallel (auto-reset off, step cap = TRAIN_STEPS); an env stops counting
after its episode ends, so the totals are the same sums.  Actions: ``training=False`` (no
Gumbel noise), the env's action mask, argmax — agilerl's eval-mode ``get_action`` restated.
Weights come from this package's safetensors checkpoints (marlnav/maddpg.py ``MADDPG.save``);
the reference's pickled ``.pt`` checkpoints are not loadable with a non-executing loader and
are not used.
"""
from __future__ import annotations

import torch

from .actor import MultiAgentActors
from .vec_env import VecGridEnv


@torch.no_grad()
def evaluate(actors: MultiAgentActors, scenario="level3", episodes: int = 100, max_steps: int = 150,
             fear: bool = False, seed: int = 42, record_actions: bool = False, fused: bool | None = None) -> dict:
    env = VecGridEnv(scenario, num_envs=episodes, fear=fear, max_steps=max_steps, auto_reset=False, seed=seed)
    fused = actors.fusable(env) if fused is None else fused
    try:
        obs, mask = env.reset()
        dev = env.device
        active = torch.ones(episodes, dtype=torch.bool, device=dev)
        crashes = torch.zeros((), dtype=torch.int64, device=dev)
        apples = torch.zeros((), dtype=torch.int64, device=dev)
        steps = torch.zeros((), dtype=torch.int64, device=dev)
        fear_sum = torch.zeros((), dtype=torch.float64, device=dev)
        recorded = []
        for i in range(max_steps):
            if fused:  # one kernel over the obs descriptors (include/actor_ops.h)
                actions, _ = actors.act_env(env, env.out["mask"], training=False)
            else:
                actions, _ = actors.act(env.out["obs"], env.out["mask"], training=False)
            if record_actions:
                recorded.append(actions.clone())
            r = env.step(actions)
            crashes += (r.crashes * active).sum()
            apples += (r.apples * active).sum()
            steps += active.sum()
            fear_sum += (r.fear.sum(1) * active).sum()
            active &= ~r.done.bool()
            # a host sync every 8 steps: stepping envs whose episode ended changes no total
            # (they are masked out), so checking late only costs the few extra steps
            if i % 8 == 7 and not bool(active.any()):
                break
        out = {"episodes": episodes, "crashes": int(crashes), "apples_caught": int(apples), "steps": int(steps),
               "fear": float(fear_sum)}
        if record_actions:
            out["actions"] = torch.stack(recorded)
        return out
    finally:
        env.close()
