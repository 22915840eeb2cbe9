"""Batched MADDPG training driver: ``MADDPGAgent.train`` (maddpg/agent.py:77-252) over the E envs
of this rank's shard, with the learner of marlnav/maddpg.py (data-parallel across ranks when a
process group exists: replicated weights, one gradient all-reduce per backward).

Per env step (all device work, no host sync):
  actor (GumbelSoftmax sample, action mask, argmax) -> gw_step (world update, FeAR, shaped
  reward, auto-reset) -> replay ring (state slot, action probabilities, shaped reward,
  termination) -> ``learns_per_step`` MADDPG updates (each the update's recorded
  launches by default, or one HIP-graph replay with ``graph=True``) once the ring holds
  ``batch_size`` transitions.

Differences from the reference loop, all structural: episodes auto-reset per env inside the
kernel instead of ``train()`` returning after one episode (``main_custom.py:129``), so one
``train(env_steps)`` call advances every env by env_steps steps; the learn schedule follows the
reference rule (``learns_per_step``) unless ``updates_per_step`` overrides it — at E >> LEARN_STEP
the rule asks for E // LEARN_STEP updates per step (6,553 at E = 65,536), which is only
practical with a larger batch, so large-E runs set it explicitly.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .maddpg import MADDPG, learns_per_step
from .rollout import Rollout
from .vec_env import VecGridEnv


def dp_env_counts(local_envs: int, device=None):
    """(global env count, smallest shard) over the default process group (one all-reduce each;
    (local_envs, local_envs) without one).  Every rank gets the same pair."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return int(local_envs), int(local_envs)
    dev = device if (device is not None and dist.get_backend() == "nccl") else torch.device("cpu")
    tot = torch.tensor([local_envs], dtype=torch.int64, device=dev)
    neg_min = torch.tensor([-local_envs], dtype=torch.int64, device=dev)
    dist.all_reduce(tot)
    dist.all_reduce(neg_min, op=dist.ReduceOp.MAX)
    return int(tot.item()), int(-neg_min.item())


def learn_schedule(idx_step: int, ring_t: int, ring_slots: int, global_envs: int, min_shard: int, learn_step: int,
                   batch_size: int, learning_delay: int = 0, updates_per_step: int | None = None) -> int:
    """MADDPG updates after env step idx_step: the reference rule (maddpg/agent.py:199-224,
    ``learns_per_step``) over the GLOBAL env count, once every rank's ring holds a batch (the
    smallest shard decides; ring_t = steps stored, the same on every rank since each rank steps
    once per step) and the transitions of all ranks exceed learning_delay.  Every input is the
    same on every rank, so every rank issues the same learn() calls (and so the same gradient
    all-reduces) even when envs % world != 0."""
    n = updates_per_step if updates_per_step is not None else learns_per_step(global_envs, learn_step, idx_step)
    filled = min(ring_t, ring_slots - 1)
    if n and filled * min_shard >= batch_size and ring_t * global_envs > learning_delay:
        return n
    return 0


class MADDPGTrainer:
    def __init__(self, env: VecGridEnv, maddpg: MADDPG, memory_size: int = 200_000, learning_delay: int = 0,
                 updates_per_step: int | None = None, graph: bool | str = "launches", seed: int = 0):
        self.env, self.m = env, maddpg
        # data parallelism: every decision that gates a learn() (and so its two gradient
        # all-reduces) is taken from GLOBAL quantities that every rank computes alike -- the global
        # env count, the smallest shard and the ring's step count (each rank steps once per step) --
        # never from this rank's shard size, which differs by one when envs % world != 0
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.world = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0
        self.global_envs, self.min_shard = dp_env_counts(env.E, env.device)
        # MEMORY_SIZE transitions in total over the ranks (each rank's ring holds its share)
        slots = max(2, -(-memory_size // self.global_envs) + 1)
        # obs writes pipelined with the next step when the actor is the fused op (it never reads
        # the dense obs), launched behind it ("lazy"); the ring is fenced before every learn
        # the learner samples the ring's rows from its obs descriptors when the actor is fused
        # (Rollout(desc_ring)): an update never waits for the obs writer of the step before it
        fusable = maddpg.actors.fusable(env)
        self.rollout = Rollout(env, maddpg.actors, replay_slots=slots, training=True, seed=seed,
                               obs_async="lazy" if fusable else False,
                               desc_ring=fusable and env.device.type == "cuda")
        self.learning_delay = learning_delay
        self.updates_per_step = updates_per_step
        # graph="launches" (default): the update re-issued as its recorded launches where every
        # launch of it goes through the C ABI (MADDPG.capture(launches=True)), else a graph replay;
        # True: always the graph replay; False: eager
        self.use_graph = bool(graph) and env.device.type == "cuda"
        self.launches = graph == "launches"
        rank = self.rollout.group_rank()
        self.gen = torch.Generator(device=env.device).manual_seed(seed + 1 + 7919 * rank)
        self.updates = 0
        self.losses = []            # (actor_loss [K], critic_loss [K]) device tensors of the last updates
        self.total_steps = 0

    def learns_now(self, idx_step: int) -> int:
        """Updates after env step idx_step (``learn_schedule``), identical on every rank."""
        rp = self.rollout.replay
        return learn_schedule(idx_step, rp.t, rp.S, self.global_envs, self.min_shard, self.m.learn_step,
                              self.m.batch_size, self.learning_delay, self.updates_per_step)

    def reset(self):
        self.rollout.reset()

    def _learn(self):
        rp = self.rollout.replay
        if self.use_graph and self.m._graph is not None and not self.m.capture_matches(rp):
            # the ring switched between descriptor and dense rows since the capture (reset after
            # load_checkpoint): the captured sample would read the other rows than the fence orders
            self.m.invalidate_capture()
        self.rollout.learn_fence()  # what the sampled transitions read (descriptor or obs slots)
        if self.use_graph:
            if self.m._graph is None:
                self.m.capture(self.rollout.replay,
                               actor_env=self.env if self.rollout.fused and not self.rollout.patch else None,
                               launches=self.launches)
            return self.m.replay_learn()
        return self.m.learn_from(self.rollout.replay, generator=self.gen)

    def train(self, env_steps: int = 150) -> dict:
        """Advance every env by env_steps steps with learning; returns the episode statistics of
        these steps (completed-episode return / length means, FeAR, crashes, apples)."""
        before = self.rollout.totals() if self.rollout.has_stats else None
        for idx_step in range(env_steps):
            self.rollout.step()
            self.total_steps += self.env.E
            n = self.learns_now(idx_step)
            if n:
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
    def _memory_file(self) -> str:
        # every rank's ring holds its own shard's transitions: one memory file per rank
        return "memory.safetensors" if self.world == 1 else f"memory_r{self.rank}.safetensors"

    def save_checkpoint(self, path: str, filename: str, steps: int | None = None):
        """The networks + optimizers (`filename`, safetensors; rank 0 writes them, the replicas
        are identical), the replay memory (`memory.safetensors`, one `memory_r<rank>` file per
        rank with data parallelism: the ring's slots, fill state and the fused actor's noise
        counter, where the reference pickles its buffer) and the step counter (`steps.txt`,
        env steps over all ranks), as the reference lays them out.  Ranks meet at a barrier
        after writing, so a load that follows sees every file."""
        import os
        from safetensors.torch import save_file
        self.rollout.fence()  # the ring's last obs slots are written
        if self.rank == 0:
            os.makedirs(path, exist_ok=True)
            self.m.save(os.path.join(path, filename))
            with open(os.path.join(path, "steps.txt"), "w") as f:
                f.write(str(self.total_steps // max(self.env.E, 1) * self.global_envs if steps is None else int(steps)))
        if self.distributed:
            dist.barrier()  # the directory exists
        if self.rollout.replay is not None:
            sd = {k: v.detach().contiguous().cpu() for k, v in self.rollout.replay.state_dict().items()}
            sd["rollout_calls"] = torch.tensor([self.rollout._calls], dtype=torch.int64)
            save_file(sd, os.path.join(path, self._memory_file()))
        if self.distributed:
            dist.barrier()

    def load_wo_memory(self, path: str, filename: str):
        """The networks and optimizers only (in place: a captured update graph stays valid; every
        rank reads rank 0's file, the replicas are identical)."""
        import os
        self.m.load(os.path.join(path, filename))

    def load_checkpoint(self, path: str, filename: str):
        import os
        from safetensors.torch import load_file
        self.load_wo_memory(path, filename)
        mem = os.path.join(path, self._memory_file())
        if self.rollout.replay is not None and os.path.exists(mem):
            self.rollout.fence()
            sd = load_file(mem)
            calls = sd.pop("rollout_calls", None)
            self.rollout.replay.load_state_dict({k: v.to(self.env.device) for k, v in sd.items()})
            # the fused actor's Gumbel-noise Philox counter continues where the saved run stopped
            # (restarting it at 0 would replay the original run's exploration noise)
            self.rollout.resume(calls=int(calls[0]) if calls is not None else None)
            self.m.invalidate_capture()  # the ring's rows now come from its dense slots: capture again
        with open(os.path.join(path, "steps.txt")) as f:
            self.total_steps = int(f.read()) // self.global_envs * self.env.E

    def total_loss(self) -> float:
        """MADDPGAgent.total_loss: sum of the most recent per-agent losses (actor + critic)."""
        if not self.losses:
            return 0.0
        a, c = self.losses[-1]
        return float(a.sum() + c.sum())
