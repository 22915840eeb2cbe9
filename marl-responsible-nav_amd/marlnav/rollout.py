"""Batched MADDPG rollout: the per-step body of MADDPGAgent.train (maddpg/agent.py:77-252) over
the E envs of this rank's shard.

Per step (all on the GPU, no host sync):
  actions, probs = actors.act(obs_t, mask_t)                 get_action          agent.py:109-122
  env.step(actions) -> obs_{t+1}, shaped reward, dones         env.step + :124-141 (in-kernel)
  replay ring <- (slot of obs_t, probs, shaped reward, term)  memory.save_to_memory :190-197
  auto-reset of done envs (in-kernel)                          the break / env.reset :241, main :129
  episode statistics added into a running total (in-kernel, gw_step_out.stats_acc)
  [multi-GPU] RCCL all-gather of every env's ep_return / done  completed_episode_scores :229-247
              (parallel.ReturnGather; the only per-step exchange)

Replay storage is zero-copy: the env writes obs_{t+1} straight into ring slot (t+1) % S, so
the obs of step t is both the next_state of transition t-1 and the state of transition t;
terminal observations of done envs go to a parallel final-obs ring (their next_state).
Learning (agilerl MADDPG.learn, agent.py:199-224) runs beside this rollout: marlnav/maddpg.py
(data-parallel across ranks) driven by marlnav/train.py or bench.py --updates-per-step.
The statistics totals are all-reduced across ranks only when read (``totals()``).
"""
from __future__ import annotations

import ctypes as C
import os

import torch
import torch.distributed as dist

from . import _lib
from .actor import MultiAgentActors
from .parallel import shard  # noqa: F401  (re-exported)
from .vec_env import VecGridEnv


class ReplayRing:
    """S steps of E transitions each, in HBM.  obs slots are written by the env directly."""

    def __init__(self, env: VecGridEnv, slots: int, patch: int = 0, desc: bool = False):
        """patch > 0: the ring holds the agents' egocentric patch x patch observations
        (VecGridEnv.obs_patch) instead of the full grids.
        desc (full-grid obs on the GPU): also keep each step's 48-byte obs descriptors per slot
        ([S][E][12] u32, 3 MB per slot at 65,536 envs); ``sample`` then expands the sampled rows
        from them (gw_replay_gather_desc, the same values bit for bit), so a learner that follows a
        step never waits for that step's obs writer.  Rollout fills it (``Rollout(desc_ring=True)``)."""
        self.S = max(2, int(slots))
        K, E, H, W, dev = env.K, env.E, env.H, env.W, env.device
        if patch:
            H = W = int(patch)
        od = env.obs_dtype if not patch else torch.float32  # bf16 obs (lossless) halves the ring
        self.obs = torch.zeros((self.S, K, E, H, W), dtype=od, device=dev)
        self.final_obs = torch.zeros((self.S, K, E, H, W), dtype=od, device=dev)
        self.probs = torch.zeros((self.S, K, E, 9), dtype=torch.float32, device=dev)
        self.reward = torch.zeros((self.S, E, K), dtype=torch.float64, device=dev)
        self.term = torch.zeros((self.S, E, K), dtype=torch.uint8, device=dev)
        self.done = torch.zeros((self.S, E), dtype=torch.uint8, device=dev)
        self.t = 0          # transitions stored = steps taken
        self.t_dev = torch.zeros((), dtype=torch.int64, device=dev)  # same, on device (graph-safe sampling)
        self.E, self.K = E, K
        self.desc = None
        self.desc_ok = False  # every descriptor slot matches its obs slot (set by Rollout.reset)
        if desc and not patch and dev.type == "cuda" and H * W <= 4096:  # (the expansion's cell limit)
            self.desc = torch.zeros((self.S, E, 12), dtype=torch.int32, device=dev)
            self._src = _lib.GwObsSource()
            _lib.check(_lib.load().gw_obs_view(env.handle, C.byref(self._src)), "gw_obs_view")
            self.env_handle = env.handle  # the env whose gw_profile spans the descriptor learner joins

    def __len__(self):
        return min(self.t, self.S - 1) * self.E

    _TENSORS = ("obs", "final_obs", "probs", "reward", "term", "done")

    def state_dict(self) -> dict:
        """The ring's contents and fill state (MADDPGAgent.save_checkpoint's memory.pkl,
        maddpg/agent.py:255-266; safetensors here, nothing is pickled)."""
        out = {n: getattr(self, n) for n in self._TENSORS}
        out["t"] = torch.tensor([self.t], dtype=torch.int64)
        out["t_dev"] = self.t_dev.reshape(1)
        return out

    @torch.no_grad()
    def load_state_dict(self, sd: dict):
        for n in self._TENSORS:
            if tuple(sd[n].shape) != tuple(getattr(self, n).shape):
                raise ValueError(f"replay ring {n}: shape {tuple(sd[n].shape)} != {tuple(getattr(self, n).shape)}")
            getattr(self, n).copy_(sd[n])
        self.t = int(sd["t"][0])
        self.t_dev.copy_(sd["t_dev"].reshape(()))
        self.desc_ok = False  # the descriptors are not saved: dense rows until the next reset

    @torch.no_grad()
    def sample(self, batch: int, generator: torch.Generator | None = None, return_idx: bool = False,
               critic_in: bool = False, extra_uniform: int = 0, philox: tuple | None = None):
        """Uniform transitions -> (state [K,B,H,W], probs [K,B,9], reward [B,K], next_state, term [B,K]).
        Every index is computed on the device from ``t_dev``, so a captured graph stays valid as
        the ring fills (MultiAgentReplayBuffer.sample, uniform without priorities).
        critic_in (GPU): also return the critic's input rows (x, x_next) that MADDPG.learn would
        build from them, from the same gather launch (x_next's action slots left to the learner)."""
        if self.t <= 0:
            raise RuntimeError("empty replay ring")
        dev = self.obs.device
        if dev.type == "cuda":
            return self._sample_hip(batch, generator, return_idx, critic_in, extra_uniform, self.use_desc, philox)
        n = torch.clamp(self.t_dev, min=1, max=self.S - 1)
        step = torch.minimum((torch.rand((batch,), device=dev, generator=generator) * n).long(), n - 1)
        env = torch.randint(0, self.E, (batch,), device=dev, generator=generator)
        tr = (self.t_dev - 1 - step) % self.S      # transition slot (its state is obs[tr])
        nx = (tr + 1) % self.S
        state = self.obs[tr, :, env].permute(1, 0, 2, 3).float()
        done = self.done[tr, env].bool()
        next_state = torch.where(done[None, :, None, None], self.final_obs[tr, :, env].permute(1, 0, 2, 3),
                                 self.obs[nx, :, env].permute(1, 0, 2, 3)).float()
        out = (state, self.probs[tr, :, env].permute(1, 0, 2), self.reward[tr, env], next_state, self.term[tr, env])
        return out + ((tr, env),) if return_idx else out

    @property
    def use_desc(self) -> bool:
        """Whether ``sample`` expands the rows from the descriptor ring (no obs-writer wait)."""
        return self.desc is not None and self.desc_ok

    def _sample_hip(self, batch, generator, return_idx, critic_in=False, extra=0, use_desc=False, philox=None):
        """sample() on the GPU: the same draws (torch.rand, then torch.randint), then the index
        arithmetic and every gather in ONE launch (gw_replay_gather, include/rollout_ops.h).
        extra > 0: that many more uniforms from the same torch.rand launch, returned last (the
        learner's Gumbel uniforms: one launch instead of three).
        philox = (seed, int32 device counter): the draws are made inside the gather launch
        (Philox keyed by seed, counter row / *counter; no torch RNG launch, so a captured update
        has no RNG bookkeeping either); returns no extra uniforms and no env indices, and with
        critic_in on the descriptor ring the state / next_state tensors come back UNWRITTEN
        (only their shapes are meaningful: the fused learner reads the critic rows)."""
        dev = self.obs.device
        if philox is not None:
            seed, ctr = int(philox[0]), philox[1]
            u = env = None
        else:
            seed, ctr = 0, None
            u_all = torch.rand((batch + int(extra),), device=dev, generator=generator)
            u = u_all[:batch]
            env = torch.randint(0, self.E, (batch,), device=dev, generator=generator)
        K, HW = self.K, self.obs.shape[-2] * self.obs.shape[-1]
        state = torch.empty((K, batch) + tuple(self.obs.shape[-2:]), device=dev, dtype=torch.float32)
        next_state = torch.empty_like(state)
        probs = torch.empty((K, batch, 9), device=dev, dtype=torch.float32)
        reward = torch.empty((batch, K), device=dev, dtype=torch.float64)
        term = torch.empty((batch, K), device=dev, dtype=torch.uint8)
        tr = torch.empty((batch,), device=dev, dtype=torch.int64) if return_idx else None
        x = xn = None
        if critic_in:
            x = torch.empty((batch, K * HW + K * 9), device=dev, dtype=torch.float32)
            xn = torch.empty_like(x)
        stream = torch.cuda.current_stream(dev).cuda_stream
        # the fused learner's in-kernel-draws path reads only the critic rows: the descriptor
        # gather then skips the [K, B, H*W] state copies (returned unwritten)
        rows_only = philox is not None and critic_in and use_desc
        outs = (None if rows_only else state.data_ptr(), None if rows_only else next_state.data_ptr(),
                probs.data_ptr(), reward.data_ptr(), term.data_ptr(),
                tr.data_ptr() if return_idx else None, x.data_ptr() if critic_in else None,
                xn.data_ptr() if critic_in else None, seed, ctr.data_ptr() if ctr is not None else None, stream)
        up = u.data_ptr() if u is not None else None
        ep = env.data_ptr() if env is not None else None
        if use_desc:
            _lib.check(_lib.load().gw_replay_gather_desc(
                C.byref(self._src), self.desc.data_ptr(), self.probs.data_ptr(), self.reward.data_ptr(),
                self.term.data_ptr(), self.done.data_ptr(), self.t_dev.data_ptr(), up, ep,
                self.S, batch, *outs), "gw_replay_gather_desc")
        else:
            _lib.check(_lib.load().gw_replay_gather(
                self.obs.data_ptr(), self.final_obs.data_ptr(), int(self.obs.dtype == torch.bfloat16),
                self.probs.data_ptr(), self.reward.data_ptr(), self.term.data_ptr(), self.done.data_ptr(),
                self.t_dev.data_ptr(), up, ep, self.S, K, self.E, HW, batch, *outs),
                "gw_replay_gather")
        out = (state, probs, reward, next_state, term)
        if return_idx:
            out = out + ((tr, env),)
        if critic_in:
            out = out + ((x, xn),)
        return out + (u_all[batch:],) if (extra and philox is None) else out


class Rollout:
    def __init__(self, env: VecGridEnv, actors: MultiAgentActors | None = None, replay_slots: int = 0,
                 training: bool = True, group=None, seed: int = 0, fused: bool | None = None,
                 obs_async: bool | str = False, fear_async: bool = False, gather=None, patch: int = 0,
                 patch_async: bool | None = None, desc_ring: bool = False):
        """fused: get_action as the one-kernel gw_actor_act over the env's obs descriptors
        (default when the actors are the f32 128-128 MLP), else the PyTorch forward over the
        dense obs with torch's Gumbel noise.
        obs_async: pipeline the env's obs writes (the replay ring's obs slots) with the next
        step's actor + world update (VecGridEnv.set_obs_async); whoever reads the obs or the ring
        afterwards calls ``fence()`` first (the learner does).
        fear_async (with obs_async): the next step's actor overlaps this step's FeAR kernel; the
        step's statistics are reduced one step later, after a FeAR fence.
        gather: a parallel.ReturnGather; every step writes its ep_return / done into the gather's
        send buffer and the completed-episode returns of all ranks are all-gathered
        (maddpg/agent.py:229-247 ``completed_episode_scores``).
        patch > 0: the actors see (and the ring stores) each agent's egocentric patch x patch
        window of its observation (VecGridEnv.obs_patch; an opt-in input format, the reference
        observes the whole grid): actors built for (H, W) = (patch, patch); the env may run
        with obs=False.
        patch_async (default: on for the CNN head, off for the MLP; GW_PATCH_ASYNC=0/1 overrides):
        with a ring and the fused actor, the window writer runs on a side stream beside the next
        step's actor (``fence()`` orders the ring slots).
        desc_ring (full-grid obs, GPU): the ring also keeps every step's obs descriptors and the
        learner samples from them (``ReplayRing(desc=True)``; ``learn_fence()`` then skips the
        obs-writer wait, so the writer of step t overlaps the updates that follow it)."""
        self.env = env
        self.actors = actors
        self.fused = (actors is not None and actors.fusable(env, patch)) if fused is None else bool(fused)
        self.seed = int(seed)
        self._calls = 0  # Philox counter of the fused path's Gumbel noise (never repeats)
        # with a replay ring the fused actor's counter is _noise_base + the ring's DEVICE step
        # count (read by the kernel at launch: graph replays draw fresh noise), which equals
        # _calls: _noise_base is _calls at the last ring reset
        self._noise_base = 0
        self._graphs = None
        self._actions = torch.empty((env.E, env.K), dtype=torch.int32, device=env.device)
        self.training = training
        self.group = group
        self.patch = int(patch)
        if self.patch and actors is not None and (actors.H, actors.W) != (self.patch, self.patch):
            raise ValueError("Rollout(patch=P) needs actors built for a P x P input")
        self.replay = ReplayRing(env, replay_slots, patch=self.patch, desc=desc_ring) if replay_slots else None
        self._patch = None  # the current obs' patches when there is no ring
        # patch windows into the ring on a side stream: the fused actor of the next step reads the
        # descriptors, not the windows, so the window writer of step t overlaps actor t+1; the
        # world update of step t+1 (which rewrites the descriptors) waits for it, and fence()
        # orders the ring slots for readers (GW_PATCH_ASYNC=0: on the caller's stream)
        if patch_async is None:  # default: on the caller's stream.  Round 3 put the CNN head's writer
            # beside it (c4patch 203 -> 184 us per step, profiles/r3_s2); since the round-5 row writer
            # (29 us alone at c4patch) the side stream costs more than it hides: its blocks take the
            # CU slots the rare kernel's two-blocks-per-CU grid needs (c4patch 156.7 beside vs 150.2
            # serial, profiles/r5_window); the MLP head's one-block-per-CU actor never gained from it
            env_pa = os.environ.get("GW_PATCH_ASYNC")
            patch_async = env_pa is not None and env_pa != "0"
        self.patch_async = (bool(patch_async) and bool(self.patch) and self.fused and self.replay is not None
                            and env.device.type == "cuda")
        if self.patch_async:
            self._pstream = torch.cuda.Stream(device=env.device)
            self._pev = torch.cuda.Event()
        self._pev_live = False
        # the CNN head on windows: the step's windows and the listing of the positions the next act
        # recomputes in ONE launch (gw_patch_cnn_write_list), then the act without its listing
        # (gw_patch_cnn_act_listed).  GW_CNN_WRITE_LIST=0: the separate writer and act (A/B)
        self._cnn_list = (self.fused and bool(self.patch) and getattr(actors, "arch", "") == "cnn" and
                          not self.patch_async and self.replay is not None and env.device.type == "cuda" and
                          env.E % 4 == 0 and os.environ.get("GW_CNN_WRITE_LIST", "1") != "0")
        self._lists_ready = False  # a listing for the env's current descriptors was launched
        self._no_list = False  # capture(): this step writes its windows without the listing
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        rank = dist.get_rank(group) if self.distributed else 0
        # the PyTorch actor's Gumbel noise: one stream per rank (the fused actor's Philox noise is
        # keyed by the global env id instead, so it is the same for any number of ranks)
        self.gen = torch.Generator(device=env.device).manual_seed(seed + 7919 * rank) if actors is not None else None
        self.t = 0
        # the step kernels add their per-block statistics rows into a running total and advance
        # the ring's device step count themselves (gw_step_out.stats_acc / tick), so a step needs
        # no reduction launch on any number of ranks; totals() all-reduces the total when read
        self._acc = torch.zeros_like(env.out["stats"]) if env.out.get("stats") is not None else None
        self.gather = gather
        if gather is not None and gather.count != env.E:
            raise ValueError("ReturnGather shard size != env.E")
        env.set_obs_async(obs_async, fear_async=fear_async)
        self._pending = None  # (stats, tick) of a step whose FeAR may still be in flight

    def group_rank(self) -> int:
        return dist.get_rank(self.group) if self.distributed else 0

    @property
    def has_stats(self) -> bool:
        """Whether the env produces the statistics rows that ``totals()`` sums."""
        return self._acc is not None

    def _flush(self):
        """Reduce the statistics of the previous step once its FeAR outputs are ordered."""
        if self._pending is not None:
            stats, tick = self._pending
            self._pending = None
            self.env.fear_fence()
            self._reduce(stats, tick)

    def _reduce(self, stats, tick):
        if self.gather is not None:
            self.gather.push()  # the step wrote ep_return / done into the gather's send buffer
        if self._acc is not None:
            return  # the step kernels accumulated the rows and advanced the tick
        if tick is not None:
            tick.add_(1)

    def _patch_join(self):
        """The current stream waits for the side stream's last window writer."""
        if self._pev_live:
            torch.cuda.current_stream(self.env.device).wait_event(self._pev)
            self._pev_live = False

    def fence(self):
        """Order everything written so far (ring slots / env obs, rewards, statistics) before
        later work on the current stream (a no-op unless obs_async or patch_async)."""
        self._patch_join()
        self._flush()
        self.env.obs_fence()

    def learn_fence(self):
        """Order what ``ReplayRing.sample`` reads before later work on the current stream: with
        the descriptor ring that is the rewards / terminations (FeAR-owned with the unjoined
        FeAR) and the descriptor slots (stream-ordered), not the obs writer; else ``fence()``."""
        if self.replay is not None and self.replay.use_desc:
            self._patch_join()
            self._flush()
        else:
            self.fence()

    def _desc_copy(self, slot: int):
        rp = self.replay
        if rp is not None and rp.desc is not None:
            _lib.check(self.env.lib.gw_obs_desc_copy(self.env.handle, rp.desc[slot].data_ptr(),
                                                      torch.cuda.current_stream(self.env.device).cuda_stream),
                       "gw_obs_desc_copy")

    def reset(self):
        # the previous step's statistics (and its ring tick) are reduced before the ring's step
        # count restarts, so t_dev never runs ahead of the transitions written
        self._patch_join()
        self._flush()
        self._lists_ready = False  # new descriptors: the next act lists itself
        if self.replay is not None:
            obs, mask = self.env.reset()
            if self.patch:
                self.env.obs_patch(self.patch, out=self.replay.obs[0])
            else:
                self.replay.obs[0].copy_(obs)
                self._desc_copy(0)
                self.replay.desc_ok = self.replay.desc is not None
            self.replay.t = 0
            self.replay.t_dev.zero_()
            self._noise_base = self._calls
            self._graphs = None
        else:
            self.env.reset()
            if self.patch and not self.fused:
                self._patch = self.env.obs_patch(self.patch, out=self._patch)
        self.t = 0

    @torch.no_grad()
    def resume(self, calls: int | None = None):
        """Continue after ReplayRing.load_state_dict: the envs start new episodes (as the reference
        does after load_checkpoint) and their first obs goes into the ring's current slot.  That
        slot was the next state of the last stored transition, so that transition keeps it as its
        terminal-obs entry (done set: sampling then reads the final-obs slot), unchanged."""
        rp = self.replay
        if rp is None:
            self.reset()
            return
        self._patch_join()
        self._flush()
        self._lists_ready = False
        t, S = rp.t, rp.S
        cur, prev = t % S, (t - 1) % S
        if t > 0:
            rp.final_obs[prev].copy_(rp.obs[cur])
            rp.done[prev].fill_(1)
        rp.desc_ok = False  # that terminal obs has no descriptor: dense rows until the next reset
        obs, _ = self.env.reset()
        if self.patch:
            self.env.obs_patch(self.patch, out=rp.obs[cur])
        else:
            rp.obs[cur].copy_(obs)
        self.t = t
        # the fused actor's noise counter continues where the saved run stopped (calls = its
        # actor calls; restarting at 0 would replay the original run's exploration noise)
        self._calls = int(calls) if calls is not None else max(self._calls, t)
        self._noise_base = self._calls - t
        self._graphs = None

    def _obs_now(self):
        if self.replay is not None:
            return self.replay.obs[self.t % self.replay.S]
        return self._patch if self.patch else self.env.out["obs"]

    @torch.no_grad()
    def step(self):
        env = self.env
        mask = env.out["mask"]
        cur = self.t % self.replay.S if self.replay is not None else 0
        if self.actors is not None and self.fused:
            probs_out = self.replay.probs[cur] if self.replay is not None else None
            if self._dev_counter():  # counter = _noise_base + t_dev (== _calls), read on the device
                actions, probs = self.actors.act_env(env, mask, self.training, seed=self.seed, counter=self._noise_base,
                                                     counter_dev=self.replay.t_dev, actions_out=self._actions,
                                                     probs_out=probs_out, patch=self.patch, listed=self._lists_ready)
            else:
                actions, probs = self.actors.act_env(env, mask, self.training, seed=self.seed, counter=self._calls,
                                                     actions_out=self._actions, probs_out=probs_out, patch=self.patch,
                                                     listed=self._lists_ready)
            self._lists_ready = False
            self._calls += 1
        elif self.actors is not None:
            if not self.patch:
                self.env.obs_fence()  # the PyTorch forward reads the dense obs
            actions, probs = self.actors.act(self._obs_now(), mask, self.training, generator=self.gen)
        else:
            actions, probs = None, None  # device-RNG random policy
        self._flush()  # after the actor: it overlapped the previous step's FeAR kernel
        if self.replay is not None:
            rp = self.replay
            nxt = (self.t + 1) % rp.S
            # zero-copy: the step writes obs_{t+1}, the terminal obs, the shaped reward and the
            # dones straight into the ring slots
            into = dict(shaped=rp.reward[cur], term=rp.term[cur], done=rp.done[cur])
            if self._acc is not None:
                into.update(stats_acc=self._acc, tick=rp.t_dev)
            if not self.patch:
                into.update(obs=rp.obs[nxt], final_obs=rp.final_obs[cur])
                if rp.desc is not None:  # the step kernels write the descriptors of slot nxt too
                    into["desc_copy"] = rp.desc[nxt]
            if self.gather is not None:
                g = self.gather.into()
                into["ep_return"] = g["ep_return"]
                # done goes to the ring slot and, from the same kernel, to the gather's send buffer
                into["done_copy"] = g["done"]
            self._patch_join()  # the previous window writer has read the descriptors
            # the step's windows inside its FeAR launch (gw_step_patch_next; FeAR on and joined):
            # the MLP head's rollout, where no listing shares the writer's launch
            step_patch = (self.patch and not self.patch_async and not self._cnn_list and env.fear_enabled and
                          not env.fear_async and env.device.type == "cuda" and
                          os.environ.get("GW_FEAR_PATCH", "1") != "0")
            if step_patch:
                env.patch_next(self.patch, rp.obs[nxt], rp.final_obs[cur])
            try:
                r = env.step(actions, into=into)
            except BaseException:
                if step_patch:  # disarm: a later gw_step must not write through these pointers
                    env.patch_next(self.patch, None, None)
                raise
            if self.patch_async:  # the step's windows, beside the next step's actor
                main = torch.cuda.current_stream(env.device)
                self._pstream.wait_stream(main)
                with torch.cuda.stream(self._pstream):
                    env.obs_patch(self.patch, final=True, out=rp.obs[nxt], final_out=rp.final_obs[cur])
                self._pev.record(self._pstream)
                self._pev_live = True
            elif self.patch and step_patch:
                pass  # written by the step (gw_step_patch_next)
            elif self.patch:  # the step's obs / terminal obs as patches, straight into the ring
                if not (self._cnn_list and not env.fear_async and not self._no_list and
                        self.actors.patch_cnn_write_list(env, self.patch, rp.obs[nxt], rp.final_obs[cur])):
                    env.obs_patch(self.patch, final=True, out=rp.obs[nxt], final_out=rp.final_obs[cur])
                else:
                    self._lists_ready = True
            if probs is not None and probs.data_ptr() != rp.probs[cur].data_ptr():
                rp.probs[cur].copy_(probs)
            rp.t = self.t + 1
        else:
            into = dict(self.gather.into()) if self.gather is not None else {}
            if self._acc is not None:
                into["stats_acc"] = self._acc
            r = env.step(actions, into=into or None)
            if self.patch and not self.fused:  # the fused actor reads the descriptors, not the windows
                self._patch = env.obs_patch(self.patch, out=self._patch)
        self.t += 1
        tick = self.replay.t_dev if self.replay is not None else None
        if self.env.fear_async:
            self._pending = (r.stats, tick)
        else:
            self._reduce(r.stats, tick)
        return r

    def _dev_counter(self) -> bool:
        """Whether the fused actor reads its noise counter from the ring's device step count:
        with a ring whose count the step kernels advance (statistics on) or that is advanced right
        after each step (FeAR joined); with the unjoined FeAR and no statistics the count is
        advanced one step late, so the host counter is used."""
        return self.replay is not None and (self._acc is not None or not self.env.fear_async)

    def capture(self, n: int) -> "RolloutGraphs":
        """Capture the rollout's steps (actor, env step, ring writes, statistics, return gather)
        as HIP graphs for the launch-bound small-batch regime (C2: 4,096 envs), where a step is
        bound by the host's launches, not by the GPU.  A step's ring slots depend on t mod S, so
        there is one graph of n steps per phase of the ring (S // n graphs, S % n == 0), replayed
        in rotation; the host-side env pipeline state each graph ends in is saved with it
        (gw_pipeline_save) and restored after its replay.  The fused actor draws its noise
        counter from the ring's device step count, so replays draw fresh noise, and a replayed
        rollout equals the eager one bit for bit (tests/test_gpu_rollout_graph.py).

        Also the local-window rollouts (patch > 0: c5patch / c4patch), whose host enqueue per step
        (the fused window actor's launches, the window writer, the env step) is about as long as
        the step itself; with patch_async the window writer forks to its side stream inside the
        graph and the graph's last writer joins before its end.

        Requirements: the fused actor, a replay ring, one rank, FeAR joined; the env's obs
        synchronous (or none: window rollouts), or async on the merged kernel path with n even
        after at least one step; a ReturnGather (if any) with window == n and nothing pending.
        Nothing runs at capture: the state is untouched until the first replay."""
        env, rp = self.env, self.replay
        if not (self.fused and rp is not None and not self.distributed and self._dev_counter()):
            raise _lib.GwError("Rollout.capture: the fused actor, a replay ring and one rank")
        if rp.S % n:
            raise _lib.GwError(f"Rollout.capture: n must divide the ring's {rp.S} slots")
        if env.obs_async and (env.kernel_path != "merged" or n % 2 or not env._obs_queued):
            raise _lib.GwError("Rollout.capture: async obs only on the merged path, an even n, after a step")
        g = self.gather
        if g is not None and (g.window != n or g._fill != 0 or g.distributed):
            raise _lib.GwError("Rollout.capture: the gather needs window == n, no pending steps and one rank")
        self._flush()
        self._patch_join()  # no side-stream writer from before the capture may be waited on inside it
        # the fused actor's workspace exists and matches the weights before the capture (a
        # derivation captured into a graph would not run for eager steps before its replay)
        self.actors.ensure_workspace(env, self.patch)
        t0, rt0, calls0 = self.t, rp.t, self._calls
        fast = getattr(self.actors, "_fast", None)
        lists0, pend0 = self._lists_ready, (fast or {}).get("pending")
        start = env.pipeline_save()
        graphs, ends = [], []
        try:
            with torch.cuda.device(env.device):
                torch.cuda.synchronize(env.device)
                for _ in range(rp.S // n):
                    cg = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(cg):
                        env.profile(False)
                        for _i in range(n):
                            # the CNN listing (gw_patch_cnn_write_list) never crosses a graph
                            # boundary: a graph's first act lists for itself and its last step
                            # writes the windows alone, so every graph replays correctly after
                            # any other graph, after eager steps and right after reset()
                            if _i == 0:
                                self._lists_ready = False
                            self._no_list = _i == n - 1
                            self.step()
                        self._patch_join()  # the graph's last window writer joins its stream
                    graphs.append(cg)
                    ends.append(env.pipeline_save())
        finally:
            # nothing ran: the host-side state is the pre-capture one
            self._no_list = False
            self.t, rp.t, self._calls = t0, rt0, calls0
            self._lists_ready = lists0
            if fast is not None:
                fast["pending"] = pend0
        env.pipeline_load(start)
        self._graphs = RolloutGraphs(self, n, graphs, ends, t0 % rp.S)
        return self._graphs

    def totals(self) -> dict:
        """Episode statistics summed over all steps (and ranks): completed-episode return sum,
        episodes, FeAR, crashes, apples, shaped reward, completed-episode length sum, env-steps.
        With several ranks this is a collective (one all-reduce of 8 doubles): every rank calls it."""
        if self._acc is None:
            return {}
        self._flush()
        local = self._acc.sum(0)
        if self.distributed:
            dist.all_reduce(local, group=self.group)
        return dict(zip(_lib.STATS_NAMES, local.cpu().tolist()))

    def completed_scores(self, last: int | None = None):
        """The completed-episode returns of every rank, oldest first (``completed_episode_scores``
        of maddpg/agent.py:229-247); needs ``gather``.  Synchronises."""
        if self.gather is None:
            raise RuntimeError("Rollout(gather=ReturnGather(...)) needed")
        self._flush()
        return self.gather.completed(last)


class RolloutGraphs:
    """The ring-phase graphs of ``Rollout.capture``: ``replay()`` advances the rollout by n steps
    with one graph launch (the graph of the current ring phase)."""

    def __init__(self, ro: Rollout, n: int, graphs: list, ends: list, phase0: int):
        self.ro, self.n, self.graphs, self.ends, self.phase0 = ro, n, graphs, ends, phase0

    def replay(self):
        ro = self.ro
        if ro._graphs is not self:
            raise RuntimeError("RolloutGraphs.replay: the rollout was reset / resumed / recaptured since the capture")
        rp = ro.replay
        off = (ro.t - self.phase0) % rp.S
        if off % self.n:
            raise RuntimeError("RolloutGraphs.replay: the rollout is not on a graph boundary (eager steps in between)")
        g = off // self.n
        self.graphs[g].replay()
        ro.env.pipeline_load(self.ends[g])
        # a graph's last step lists nothing and its acts leave the bucket counters zeroed (capture)
        ro._lists_ready = False
        fast = getattr(ro.actors, "_fast", None)
        if fast is not None:
            fast["pending"] = False
        ro.t += self.n
        rp.t = ro.t
        ro._calls += self.n
