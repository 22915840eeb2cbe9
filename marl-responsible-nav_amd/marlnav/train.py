"""Batched MADDPG training driver: ``MADDPGAgent.train`` (maddpg/agent.py:77-252) over the E envs
of this rank's shard, with the learner of marlnav/maddpg.py (data-parallel across ranks when a
process group exists: replicated weights, one gradient all-reduce per backward).

Per env step (all device work, no host sync):
  actor (GumbelSoftmax sample, action mask, argmax) -> gw_step (world update, FeAR, shaped
  reward, auto-reset) -> replay ring (state slot, action probabilities, shaped reward,
  termination) -> ``learns_per_step`` MADDPG updates (one HIP-graph replay each when
  ``graph=True``) once the ring holds ``batch_size`` transitions.

Differences from the reference loop, all structural: episodes auto-reset per env inside the
kernel instead of ``train()`` returning after one episode (``main_custom.py:129``), so one
``train(env_steps)`` call advances every env by env_steps steps; the learn schedule follows the
reference rule (``learns_per_step``) unless ``updates_per_step`` overrides it — at E >> LEARN_STEP
the rule asks for E // LEARN_STEP updates per step (6,553 at E = 65,536), which is only
practical with a larger batch, so large-E runs set it explicitly.
"""
from __future__ import annotations

import torch

from .maddpg import MADDPG, learns_per_step
from .rollout import Rollout
from .vec_env import VecGridEnv


class MADDPGTrainer:
    def __init__(self, env: VecGridEnv, maddpg: MADDPG, memory_size: int = 200_000, learning_delay: int = 0,
                 updates_per_step: int | None = None, graph: bool = True, seed: int = 0):
        self.env, self.m = env, maddpg
        slots = max(2, -(-memory_size // env.E) + 1)
        # obs writes pipelined with the next step when the actor is the fused op (it never reads
        # the dense obs), launched behind it ("lazy"); the ring is fenced before every learn
        self.rollout = Rollout(env, maddpg.actors, replay_slots=slots, training=True, seed=seed,
                               obs_async="lazy" if maddpg.actors.fusable(env) else False)
        self.learning_delay = learning_delay
        self.updates_per_step = updates_per_step
        self.use_graph = graph and env.device.type == "cuda"
        rank = self.rollout.group_rank()
        self.gen = torch.Generator(device=env.device).manual_seed(seed + 1 + 7919 * rank)
        self.updates = 0
        self.losses = []            # (actor_loss [K], critic_loss [K]) device tensors of the last updates
        self.total_steps = 0

    def reset(self):
        self.rollout.reset()

    def _learn(self):
        self.rollout.fence()  # the sampled transitions read the ring's obs slots
        if self.use_graph:
            if self.m._graph is None:
                self.m.capture(self.rollout.replay)
            return self.m.replay_learn()
        return self.m.learn_from(self.rollout.replay, generator=self.gen)

    def train(self, env_steps: int = 150) -> dict:
        """Advance every env by env_steps steps with learning; returns the episode statistics of
        these steps (completed-episode return / length means, FeAR, crashes, apples)."""
        rp = self.rollout.replay
        before = self.rollout.totals() if self.rollout.has_stats else None
        for idx_step in range(env_steps):
            self.rollout.step()
            self.total_steps += self.env.E
            n = self.updates_per_step if self.updates_per_step is not None else \
                learns_per_step(self.env.E, self.m.learn_step, idx_step)
            if n and len(rp) >= self.m.batch_size and rp.t * self.env.E > self.learning_delay:
                for _ in range(n):
                    out = self._learn()
                    self.updates += 1
                self.losses = [tuple(t.clone() for t in out)]
        tot = self.rollout.totals() if self.rollout.has_stats else {}
        if before:
            tot = {k: v - before.get(k, 0.0) for k, v in tot.items()}
        eps = max(tot.get("episodes", 0.0), 1.0)
        return {"env_steps": self.total_steps, "updates": self.updates,
                "mean_return": tot.get("done_return", 0.0) / eps, "mean_len": tot.get("done_len", 0.0) / eps,
                "episodes": tot.get("episodes", 0.0), "fear": tot.get("fear", 0.0),
                "crashes": tot.get("crashes", 0.0), "apples": tot.get("apples", 0.0)}

    # ---- MADDPGAgent.save_checkpoint / load_checkpoint / load_wo_memory (maddpg/agent.py:255-281)
    def save_checkpoint(self, path: str, filename: str, steps: int | None = None):
        """The networks + optimizers (`filename`, safetensors), the replay memory
        (`memory.safetensors`: the ring's slots and fill state, where the reference pickles its
        buffer) and the step counter (`steps.txt`), as the reference lays them out."""
        import os
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        self.rollout.fence()  # the ring's last obs slots are written
        self.m.save(os.path.join(path, filename))
        if self.rollout.replay is not None:
            save_file({k: v.detach().contiguous().cpu() for k, v in self.rollout.replay.state_dict().items()},
                      os.path.join(path, "memory.safetensors"))
        with open(os.path.join(path, "steps.txt"), "w") as f:
            f.write(str(self.total_steps if steps is None else int(steps)))

    def load_checkpoint(self, path: str, filename: str):
        import os
        from safetensors.torch import load_file
        self.load_wo_memory(path, filename)
        mem = os.path.join(path, "memory.safetensors")
        if self.rollout.replay is not None and os.path.exists(mem):
            self.rollout.fence()
            self.rollout.replay.load_state_dict({k: v.to(self.env.device) for k, v in load_file(mem).items()})
            self.rollout.resume()
        with open(os.path.join(path, "steps.txt")) as f:
            self.total_steps = int(f.read())

    def load_wo_memory(self, path: str, filename: str):
        """The networks and optimizers only (in place: a captured update graph stays valid)."""
        import os
        self.m.load(os.path.join(path, filename))

    def total_loss(self) -> float:
        """MADDPGAgent.total_loss: sum of the most recent per-agent losses (actor + critic)."""
        if not self.losses:
            return 0.0
        a, c = self.losses[-1]
        return float(a.sum() + c.sum())
