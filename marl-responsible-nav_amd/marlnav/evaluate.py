"""Evaluation driver: ``customeval.py:70-133`` batched.

The reference evaluates a trained MADDPG for ``eval_episodes = 100`` episodes, one env at a
time: every episode runs at most TRAIN_STEPS steps (``configs/custom.yaml``) and stops when all
RL agents are terminated or all are truncated; it sums ``info["agent_crashes"]`` and
``info["apples_caught"]`` over all steps taken and counts the steps.  Here the episodes run as
E = episodes envs in parallel (auto-reset off, step cap = TRAIN_STEPS); an env stops counting
after its episode ends, so the totals are the same sums.  Actions: ``training=False`` (no
Gumbel noise), the env's action mask, argmax — agilerl's eval-mode ``get_action`` restated.
With the fused actor the env writes no dense obs (the actor reads the obs descriptors).
Weights come from this package's safetensors checkpoints (marlnav/maddpg.py ``MADDPG.save``) or
from the reference's shipped agilerl ``.pt`` checkpoints, read without unpickling by
marlnav/checkpoint.py (``agents.load_wo_memory``, maddpg/agent.py:279-281); those are
single-agent actors (obs 160 = Level 3's 10 x 16), evaluated on the single-agent CustomEnv
(``variant=1``, custom/customenv.py:78-183).
"""
from __future__ import annotations

from types import SimpleNamespace

import torch

from . import _lib
from .actor import MultiAgentActors
from .scenario import builtin
from .vec_env import VecGridEnv


@torch.no_grad()
def evaluate(actors: MultiAgentActors, scenario="level3", episodes: int = 100, max_steps: int = 150,
             fear: bool = False, seed: int = 42, record_actions: bool = False, fused: bool | None = None,
             variant: int = 0) -> dict:
    sc = builtin(scenario) if isinstance(scenario, str) else scenario
    if fused is None:
        fused = actors.fusable(SimpleNamespace(K=sc.K, H=sc.H, W=sc.W))
    # the fused actor reads the obs descriptors: no dense obs is written at all
    env = VecGridEnv(sc, num_envs=episodes, fear=fear, max_steps=max_steps, auto_reset=False, seed=seed,
                     obs=not fused, variant=variant)
    try:
        obs, mask = env.reset()
        dev = env.device
        active = torch.ones(episodes, dtype=torch.uint8, device=dev)
        counts = torch.zeros(3, dtype=torch.int64, device=dev)       # crashes, apples, steps
        fear_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        lib = _lib.load()
        recorded = []
        alive = torch.zeros(max_steps, dtype=torch.bool, device=dev) if record_actions else None
        for i in range(max_steps):
            if fused:  # one kernel over the obs descriptors (include/actor_ops.h)
                actions, _ = actors.act_env(env, env.out["mask"], training=False)
            else:
                actions, _ = actors.act(env.out["obs"], env.out["mask"], training=False)
            if record_actions:
                recorded.append(actions.clone())
            r = env.step(actions)
            # the active envs' crashes, apples, steps and FeAR summed, then the done ones retired
            _lib.check(lib.gw_eval_accum(r.crashes.data_ptr(), r.apples.data_ptr(), r.fear.data_ptr(),
                                         r.done.data_ptr(), active.data_ptr(), counts.data_ptr(), fear_sum.data_ptr(),
                                         episodes, env.K, torch.cuda.current_stream(dev).cuda_stream),
                       "gw_eval_accum")
            if record_actions:
                alive[i] = active.any()  # device-side: is any episode still running after step i
            # a host sync every 8 steps: stepping envs whose episode ended changes no total
            # (they are masked out), so checking late only costs the few extra steps
            if i % 8 == 7 and not bool(active.any()):
                break
        c = counts.tolist()
        out = {"episodes": episodes, "crashes": c[0], "apples_caught": c[1], "steps": c[2], "fear": float(fear_sum)}
        if record_actions:
            # the early-stop check runs every 8 steps: keep the actions up to the first step after
            # which every episode had ended (the steps an env-at-a-time loop would have taken)
            n = len(recorded)
            dead = (~alive[:n]).nonzero()
            if dead.numel():
                n = int(dead[0, 0]) + 1
            out["actions"] = torch.stack(recorded[:n])
        return out
    finally:
        env.close()
