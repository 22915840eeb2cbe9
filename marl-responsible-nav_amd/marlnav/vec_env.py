"""VecGridEnv: E independent CustomMAEnv episodes resident on one MI355X.

Tensor API over libgridenv (include/gridenv.h).  One ``step`` is the reference's
``CustomMAEnv.step`` (custom/ma_customenv.py:217-334) applied to all E envs at once, plus the
per-step reward/score arithmetic of ``MADDPGAgent.train`` (maddpg/agent.py:124-173) and an
optional auto-reset (the ``break`` + ``env.reset()`` of maddpg/agent.py:241 / main_custom.py:129).

Layouts (device tensors, owned by the env and overwritten by the next call):
  obs        [K, E, H, W] float32   agent-major: obs[k] is RL agent k's actor input batch
             (obs_dtype=torch.bfloat16: the same values, exact, in half the bytes)
  reward, fear, shaped      [E, K] float64
  term, trunc               [E, K] uint8;  done [E] uint8
  mask       [E, K] int16 (9-bit action mask, bit a = action a allowed)
  crashes, apples, ep_len   [E] int32;  ep_return, ep_fear [E] float64
  debug outputs (debug=True): actions/mdr/final_pos [E, N] int32, crash_bits/restr_bits [E] uint8
  stats (stats=True): [rows, 8] float64 per-block partial sums of the step (_lib.STATS_NAMES)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .scenario import CompiledScenario, builtin


@dataclass
class StepResult:
    obs: torch.Tensor
    reward: torch.Tensor
    fear: torch.Tensor
    shaped: torch.Tensor
    term: torch.Tensor
    trunc: torch.Tensor
    done: torch.Tensor
    mask: torch.Tensor
    crashes: torch.Tensor
    apples: torch.Tensor
    ep_return: torch.Tensor
    ep_fear: torch.Tensor
    ep_len: torch.Tensor
    final_obs: torch.Tensor | None = None
    actions: torch.Tensor | None = None
    mdr: torch.Tensor | None = None
    final_pos: torch.Tensor | None = None
    crash_bits: torch.Tensor | None = None
    restr_bits: torch.Tensor | None = None
    stats: torch.Tensor | None = None   # [rows, 8] per-block partial sums (_lib.STATS_NAMES)
    done_copy: torch.Tensor | None = None  # a second destination of done (step(into=...))
    stats_acc: torch.Tensor | None = None  # running per-block totals (step(into=...))
    tick: torch.Tensor | None = None       # += 1 per step (step(into=...))
    desc_copy: torch.Tensor | None = None  # [E, 12] int32 copy of the obs descriptors (step(into=...))


class StepGraph:
    """n captured VecGridEnv.step calls (VecGridEnv.capture_steps); replay() advances every env by
    n steps with one graph launch on the current stream."""

    def __init__(self, env, graph: torch.cuda.CUDAGraph):
        self.env, self.graph = env, graph

    def replay(self):
        self.graph.replay()
        self.env._replayed()


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous()
    return t.data_ptr()


class VecGridEnv:
    def __init__(self, scenario: CompiledScenario | str = "level3", num_envs: int = 1, fear: bool = True,
                 fear_weight: float = -5.0, max_steps: int = 150, auto_reset: bool = True, seed: int = 42,
                 device: torch.device | int | None = None, env_offset: int = 0, final_obs: bool = False,
                 debug: bool = False, obs: bool = True, stats: bool = False, variant: int | str = 0,
                 obs_dtype: torch.dtype = torch.float32):
        if not torch.cuda.is_available():
            raise _lib.GwError("VecGridEnv needs a HIP device (no CPU fallback by design)")
        sc = builtin(scenario) if isinstance(scenario, str) else scenario
        self.sc = sc
        self.E = int(num_envs)
        self.N, self.K, self.H, self.W = sc.N, sc.K, sc.H, sc.W
        self.fear_enabled = bool(fear)
        self.fear_weight = float(fear_weight)
        self.max_steps = int(max_steps)
        self.auto_reset = bool(auto_reset)
        self.seed = int(seed)
        # 0 / "multi": CustomMAEnv;  1 / "single": the single-agent CustomEnv (custom/customenv.py)
        self.variant = {"multi": 0, "single": 1}.get(variant, variant) if isinstance(variant, str) else int(variant)
        self.env_offset = int(env_offset)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   (device if isinstance(device, int) else device.index or 0))
        self.lib = _lib.load()

        keep = dict(region=np.ascontiguousarray(sc.region, np.uint8),
                    policy_id=np.ascontiguousarray(sc.policy_id, np.uint8),
                    cdf=np.ascontiguousarray(sc.policy_cdf, np.float64),
                    mdr=np.ascontiguousarray(sc.mdr, np.uint8),
                    apples=np.ascontiguousarray(sc.apples, np.int32))
        scn = _lib.GwScenario(sc.H, sc.W, keep["region"].ctypes.data, keep["policy_id"].ctypes.data,
                              int(sc.policy_cdf.shape[0]), keep["cdf"].ctypes.data, keep["mdr"].ctypes.data,
                              keep["apples"].ctypes.data)
        cfg = _lib.GwConfig(self.N, self.K, self.E, self.env_offset, int(self.fear_enabled), self.fear_weight,
                            self.max_steps, int(self.auto_reset), self.seed & 0xFFFFFFFFFFFFFFFF, self.variant)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_create(C.byref(scn), C.byref(cfg), self.device.index, C.byref(h)), "gw_create")
        self.handle = h
        if obs_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("obs_dtype: torch.float32 or torch.bfloat16")
        self.obs_dtype = obs_dtype
        if obs_dtype == torch.bfloat16:  # lossless: every obs value is exact in bf16
            _lib.check(self.lib.gw_set_obs_dtype(self.handle, 1), "gw_set_obs_dtype")
        if not obs and self.fear_enabled:
            # no full-obs writer to overlap: FeAR is on the step's critical path, where twice the
            # resident waves (32-env blocks) are faster (the local-window rollouts, profiles/r6_ab)
            _lib.check(self.lib.gw_set_fear_blocks(self.handle, 0), "gw_set_fear_blocks")

        dev, E, K, N = self.device, self.E, self.K, self.N
        f64 = dict(dtype=torch.float64, device=dev)
        self.out = dict(
            obs=torch.empty((K, E, sc.H, sc.W), dtype=obs_dtype, device=dev) if obs else None,
            final_obs=torch.full((K, E, sc.H, sc.W), float("nan"), dtype=obs_dtype, device=dev) if final_obs else None,
            reward=torch.zeros((E, K), **f64), fear=torch.zeros((E, K), **f64), shaped=torch.zeros((E, K), **f64),
            term=torch.zeros((E, K), dtype=torch.uint8, device=dev),
            trunc=torch.zeros((E, K), dtype=torch.uint8, device=dev),
            done=torch.zeros(E, dtype=torch.uint8, device=dev),
            mask=torch.zeros((E, K), dtype=torch.int16, device=dev),
            crashes=torch.zeros(E, dtype=torch.int32, device=dev),
            apples=torch.zeros(E, dtype=torch.int32, device=dev),
            ep_return=torch.zeros(E, **f64), ep_fear=torch.zeros(E, **f64),
            ep_len=torch.zeros(E, dtype=torch.int32, device=dev),
            actions=torch.zeros((E, N), dtype=torch.int32, device=dev) if debug else None,
            mdr=torch.zeros((E, N), dtype=torch.int32, device=dev) if debug else None,
            final_pos=torch.zeros((E, N), dtype=torch.int32, device=dev) if debug else None,
            crash_bits=torch.zeros(E, dtype=torch.uint8, device=dev) if debug else None,
            restr_bits=torch.zeros(E, dtype=torch.uint8, device=dev) if debug else None,
            stats=torch.zeros((int(self.lib.gw_stats_rows(self.handle)), _lib.GW_STATS), **f64) if stats else None,
            done_copy=None, stats_acc=None, tick=None, desc_copy=None,
        )
        self._step_out = _lib.GwStepOut(*[_ptr(self.out[n]) for n in _lib.STEP_OUT_FIELDS])
        self._into_cache = {}  # step(): (GwStepOut, fields, StepResult) per set of destination buffers
        self._into_sizes = None  # the destination sizes step(into=...) checks (built on first use)
        self._dev_index = self.device.index
        self._closed = False
        self._obs_queued = False  # async obs: the last step's writer not yet launched / fenced
        self.obs_async = False
        self.fear_async = False
        # the kernel path gw_create picked (GW_KERNEL, or by batch size: gw_kernel_path)
        self.kernel_path = ("v1", "split", "fused", "defer", "merged")[int(self.lib.gw_kernel_path(self.handle))]
        self.fused = self.kernel_path == "fused"

    # ------------------------------------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def reset(self, spawn: torch.Tensor | None = None, env_mask: torch.Tensor | None = None):
        """CustomMAEnv.reset for all envs (or those with env_mask != 0).
        spawn: [E, N] int32 sorted road cells (replay) or None (device RNG)."""
        spawn = self._as_i32(spawn, (self.E, self.N))
        if env_mask is not None:
            env_mask = env_mask.to(device=self.device, dtype=torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_reset(self.handle, _ptr(env_mask), _ptr(spawn), _ptr(self.out["obs"]),
                                         _ptr(self.out["mask"]), self._stream()), "gw_reset")
        self._obs_queued = False
        return self.out["obs"], self.out["mask"]

    _INTO_SPEC = {"obs": (torch.float32, "KEHW"), "final_obs": (torch.float32, "KEHW"),
                  "reward": (torch.float64, "EK"), "fear": (torch.float64, "EK"), "shaped": (torch.float64, "EK"),
                  "term": (torch.uint8, "EK"), "trunc": (torch.uint8, "EK"), "done": (torch.uint8, "E"),
                  "done_copy": (torch.uint8, "E"), "stats_acc": (torch.float64, "ROWS"),
                  "tick": (torch.int64, "ONE"), "desc_copy": (torch.int32, "DESC"),
                  "ep_return": (torch.float64, "E")}

    def step(self, rl_actions: torch.Tensor | None = None, scripted: torch.Tensor | None = None,
             spawn: torch.Tensor | None = None, obs_out: torch.Tensor | None = None,
             final_obs_out: torch.Tensor | None = None, into: dict | None = None) -> StepResult:
        """rl_actions [E, K] int32 (None = uniform random RL policy on device);
        scripted [E, N-K] (replay) or None (scenario policy on device);
        spawn [E, N] spawns for auto-resetting envs (replay) or None;
        obs_out / final_obs_out: [K, E, H, W] float32 buffers to write this step's obs into
        instead of the env's own (e.g. a replay-ring slot: zero-copy replay storage);
        into: the same for any of obs, final_obs, reward, fear, shaped, term, trunc, done,
        done_copy (a second destination of done), ep_return, stats_acc (per-block rows every
        step ADDS to: a running total), tick (int64 scalar, += 1 per step) (contiguous tensors of
        the output's dtype and size; e.g. the send buffer of parallel.ReturnGather)."""
        rl = self._as_i32(rl_actions, (self.E, self.K))
        sa = self._as_i32(scripted, (self.E, self.N - self.K))
        sp = self._as_i32(spawn, (self.E, self.N))
        over = dict(into or {})
        if obs_out is not None:
            over["obs"] = obs_out
        if final_obs_out is not None:
            over["final_obs"] = final_obs_out
        # the step's output struct and result per set of destination buffers, built once: a
        # pipelined step's host enqueue is on the critical path of short runs (the first step)
        key = tuple((n, t.data_ptr(), t.dtype, t.numel()) for n, t in over.items())
        cached = self._into_cache.get(key)
        if cached is None:
            cached = self._build_into(over)
            if len(self._into_cache) >= 4096:
                self._into_cache.clear()
            self._into_cache[key] = cached
        so, res, result = cached
        if torch.cuda.current_device() != self._dev_index:
            with torch.cuda.device(self.device):
                _lib.check(self.lib.gw_step(self.handle, _ptr(rl), _ptr(sa), _ptr(sp), C.byref(so),
                                            self._stream()), "gw_step")
        else:
            _lib.check(self.lib.gw_step(self.handle, _ptr(rl), _ptr(sa), _ptr(sp), C.byref(so),
                                        torch.cuda.current_stream().cuda_stream), "gw_step")
        self._obs_queued = self.obs_async and (res["obs"] is not None or res["final_obs"] is not None)
        return result

    def _build_into(self, over: dict):
        """(GwStepOut, result fields, StepResult) for the destination buffers ``over``."""
        so = self._step_out
        res = self.out
        if over:
            so = _lib.GwStepOut.from_buffer_copy(self._step_out)
            res = dict(self.out)
            sizes = self._into_sizes
            if sizes is None:
                sizes = self._into_sizes = {"KEHW": self.K * self.E * self.H * self.W, "EK": self.E * self.K,
                                            "E": self.E, "ONE": 1, "DESC": self.E * 12,
                                            "ROWS": int(self.lib.gw_stats_rows(self.handle)) * _lib.GW_STATS}
            for name, t in over.items():
                dt, shp = self._INTO_SPEC[name]
                if shp == "KEHW":
                    dt = self.obs_dtype
                if t.dtype != dt or t.numel() != sizes[shp] or not t.is_contiguous() or t.device != self.device:
                    raise ValueError(f"step(into={name!r}): need a contiguous {dt} tensor of {sizes[shp]} elements "
                                     f"on {self.device}")
                setattr(so, name, _ptr(t))
                res[name] = t
        return so, res, StepResult(**res)

    def capture_steps(self, n: int, gather=None) -> "StepGraph":
        """Capture ``n`` consecutive ``step()`` calls (device RNG policies, no host inputs) into
        one HIP graph; each ``replay()`` then advances every env by n steps with a single launch
        from the host.  For the small-E regime, where a step is bound by its launch chain
        (C2: 4,096 envs), not by the GPU.  Nothing runs at capture time: the env's state is
        untouched until the first replay.

        gather: a parallel.ReturnGather with ``window == n`` and no steps pending (one rank):
        each captured step writes its returns into the gather's next slot and the window is
        compacted at the end of the graph, so every replay leaves the gather as it found it.
        HIP timing events cannot be recorded in a graph: profiling is switched off for the capture.

        Synchronous obs, or async obs on the merged kernel path: there every step is ONE
        step_obs launch (step t + the obs writer of step t-1, no events), so a capture of an EVEN
        number of steps that starts with the previous step's writer queued (at least one step
        since the last reset / fence, writing the same obs buffers as the captured steps) ends
        in the state it started from, and replays chain.  The defer path's async pipeline
        (cross-queue events between steps) cannot be captured."""
        if self.obs_async:
            if self.kernel_path != "merged":
                raise _lib.GwError("capture_steps: synchronous obs, or async obs on the merged path only")
            if n % 2 or not self._obs_queued:
                raise _lib.GwError("capture_steps (merged async obs): an even n, after a step (the previous "
                                   "step's obs writer queued)")
        if gather is not None and (gather.window != n or gather._fill != 0 or gather.distributed):
            raise _lib.GwError("capture_steps: the gather needs window == n, no pending steps and one rank")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            with torch.cuda.graph(g):
                self.profile(False)
                for i in range(n):
                    self.step(into=gather.into() if gather is not None else None)
                    if gather is not None:
                        gather.push()
        return StepGraph(self, g)

    def pipeline_save(self) -> bytes:
        """The host-side pipeline state (gw_pipeline_save): after capturing a graph of steps."""
        lib = self.lib
        buf = (C.c_char * int(lib.gw_pipeline_state_bytes()))()
        _lib.check(lib.gw_pipeline_save(self.handle, buf), "gw_pipeline_save")
        return bytes(buf)

    def pipeline_load(self, state: bytes, queued: bool | None = None):
        """Restore a pipeline_save state (after replaying the graph it was saved for; the next
        queued writer then runs on the current stream)."""
        buf = (C.c_char * len(state)).from_buffer_copy(state)
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_pipeline_load(self.handle, buf, self._stream()), "gw_pipeline_load")
        self._obs_queued = self.obs_async if queued is None else bool(queued)

    def _replayed(self):
        """Host-side pipeline state after a StepGraph replay (gw_graph_replayed)."""
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_graph_replayed(self.handle, self._stream()), "gw_graph_replayed")
        self._obs_queued = self.obs_async

    def _as_i32(self, t, shape):
        if t is None:
            return None
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t))
        t = t.to(device=self.device, dtype=torch.int32).contiguous()
        if tuple(t.shape) != tuple(shape):
            t = t.reshape(shape)
        return t

    # ------------------------------------------------------------------------------------
    def state(self) -> dict:
        """Copy of the env state (device tensors): pos [N, E] cells, flags, t, episode,
        prev_dist [K, E], score, fear_score."""
        E, N, K, dev = self.E, self.N, self.K, self.device
        st = dict(pos=torch.empty((N, E), dtype=torch.int32, device=dev),
                  flags=torch.empty(E, dtype=torch.int32, device=dev),
                  t=torch.empty(E, dtype=torch.int32, device=dev),
                  episode=torch.empty(E, dtype=torch.int32, device=dev),
                  prev_dist=torch.empty((K, E), dtype=torch.int32, device=dev),
                  score=torch.empty(E, dtype=torch.float64, device=dev),
                  fear_score=torch.empty(E, dtype=torch.float64, device=dev))
        gs = _lib.GwState(*[_ptr(st[n]) for n in _lib.STATE_FIELDS])
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_copy_state(self.handle, C.byref(gs), 0, self._stream()), "gw_copy_state")
        return st

    def set_state(self, st: dict):
        gs = _lib.GwState(*[_ptr(st[n].contiguous()) if st.get(n) is not None else None
                            for n in _lib.STATE_FIELDS])
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_copy_state(self.handle, C.byref(gs), 1, self._stream()), "gw_copy_state")

    def fear_matrix(self, cells, actions, mdr=None, in_list=None) -> dict:
        """Responsibility.FeAR (full N x N matrix) and FeAL for n world snapshots of this env's map
        (gw_fear_matrix): cells / actions [n, N], mdr [n, N] or None (per-cell MdR), in_list [n]
        N-bit masks of the agents in ActionID4Agents or None (all).  -> device tensors resp
        [n, N, N] f64, vm, va [n, N, N] i32, feal [n, N] f64, feal_vm, feal_va [n, N] i32."""
        cells = torch.as_tensor(cells, device=self.device).to(torch.int32).contiguous()
        n, N = cells.shape[0], self.N
        assert cells.shape == (n, N)
        acts = self._as_i32(actions, (n, N))
        mdr = self._as_i32(mdr, (n, N))
        if in_list is not None:
            in_list = torch.as_tensor(in_list, device=self.device).to(torch.uint8).contiguous().reshape(n)
        dev = self.device
        out = dict(resp=torch.empty((n, N, N), dtype=torch.float64, device=dev),
                   vm=torch.empty((n, N, N), dtype=torch.int32, device=dev),
                   va=torch.empty((n, N, N), dtype=torch.int32, device=dev),
                   feal=torch.empty((n, N), dtype=torch.float64, device=dev),
                   feal_vm=torch.empty((n, N), dtype=torch.int32, device=dev),
                   feal_va=torch.empty((n, N), dtype=torch.int32, device=dev))
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_fear_matrix(self.handle, n, _ptr(cells), _ptr(acts), _ptr(mdr), _ptr(in_list),
                                               *[_ptr(out[k]) for k in ("resp", "vm", "va", "feal", "feal_vm",
                                                                         "feal_va")], self._stream()),
                       "gw_fear_matrix")
        return out

    def obs_patch(self, size: int, final: bool = False, out: torch.Tensor | None = None,
                  final_out: torch.Tensor | None = None):
        """Egocentric local observations (gw_obs_patch): [K, E, size, size] float32, agent k's obs
        cropped to the size x size window centred on its own cell, cells outside the grid -1.
        An opt-in input format (the reference observes the whole grid); derived from the obs
        descriptors, so the env may run without dense obs (``obs=False``).  final=True also
        returns the terminal-obs patches of the envs done at the last step: (patch, final)."""
        K, E, P = self.K, self.E, int(size)
        if out is None:
            out = torch.empty((K, E, P, P), dtype=torch.float32, device=self.device)
        if final and final_out is None:
            final_out = torch.full((K, E, P, P), float("nan"), dtype=torch.float32, device=self.device)
        for t in (out, final_out):
            if t is not None and (t.dtype != torch.float32 or t.numel() != K * E * P * P or not t.is_contiguous()):
                raise ValueError(f"obs_patch: need contiguous float32 [K, E, {P}, {P}] buffers")
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_obs_patch(self.handle, P, _ptr(out), _ptr(final_out) if final else None,
                                             self._stream()), "gw_obs_patch")
        return (out, final_out) if final else out

    def patch_next(self, size: int, out: torch.Tensor, final_out: torch.Tensor | None = None):
        """Have the next ``step`` write its P x P windows into ``out`` / ``final_out`` exactly as
        ``obs_patch(size, final=True, out=out, final_out=final_out)`` right after it would
        (gw_step_patch_next): with FeAR on, inside the FeAR launch where the row writer applies."""
        K, E, P = self.K, self.E, int(size)
        for t in (out, final_out):
            if t is not None and (t.dtype != torch.float32 or t.numel() != K * E * P * P or not t.is_contiguous()):
                raise ValueError(f"patch_next: need contiguous float32 [K, E, {P}, {P}] buffers")
        _lib.check(self.lib.gw_step_patch_next(self.handle, P, _ptr(out), _ptr(final_out)), "gw_step_patch_next")

    def set_obs_async(self, enable: bool | str = True, fear_async: bool = False):
        """Pipeline the obs writer of step t with the world update of step t+1 (gw_set_obs_async).
        While on, ``step``'s obs / final_obs are ready on the current stream only after
        ``obs_fence()`` (rewards, dones, masks and state are ordered as usual).
        enable="lazy": the writer is launched at the next step, behind the caller's work between
        the steps (an actor kernel), instead of right after the world update.
        fear_async (defer path, FeAR on): the FeAR-owned outputs (fear, shaped, ep_return,
        ep_fear, the FeAR stats rows) are ready only after ``fear_fence()``, so the caller's next
        work (the fused actor) overlaps the FeAR kernel."""
        mode = 2 if enable == "lazy" else int(bool(enable))
        if mode and fear_async:
            mode |= 4
        _lib.check(self.lib.gw_set_obs_async(self.handle, mode), "gw_set_obs_async")
        if not mode:
            self._obs_queued = False
        self.obs_async = bool(mode)
        self.fear_async = bool(mode & 4)

    def obs_fence(self):
        """Order the last step's outputs (obs, and FeAR-owned ones) before later work on the
        current stream (async mode)."""
        if self.obs_async:
            with torch.cuda.device(self.device):
                _lib.check(self.lib.gw_obs_fence(self.handle, self._stream()), "gw_obs_fence")
            self._obs_queued = False

    def fear_fence(self):
        """Order the last step's FeAR-owned outputs before later work on the current stream."""
        if self.fear_async:
            with torch.cuda.device(self.device):
                _lib.check(self.lib.gw_fear_fence(self.handle, self._stream()), "gw_fear_fence")

    def profile(self, enable: bool = True, reserve: int = 0):
        """Time each gw_step kernel with HIP events (see gw_profile); reserve: create that many
        timing events now, outside any timed region."""
        _lib.check(self.lib.gw_profile(self.handle, max(int(enable), int(reserve)) if enable else 0), "gw_profile")

    def count_sims(self, counter: torch.Tensor | None):
        """Count the FeAR counterfactual world updates (de-duplicated sims, gw_count_sims) of the
        following steps into ``counter`` (int64 [1] on the env's device; None stops counting)."""
        if counter is not None:
            assert counter.dtype == torch.int64 and counter.device == self.device and counter.numel() >= 1
        _lib.check(self.lib.gw_count_sims(self.handle, counter.data_ptr() if counter is not None else None),
                   "gw_count_sims")

    def profile_spans(self):
        """-> float64 [n, 3] (kind, start ms, end ms) of every timed launch since the last
        profile_read (gw_profile_spans; call before profile_read, which clears them)."""
        import numpy as np
        n = C.c_int64()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_profile_spans(self.handle, None, 0, C.byref(n)), "gw_profile_spans")
            buf = (C.c_double * (3 * max(n.value, 1)))()
            _lib.check(self.lib.gw_profile_spans(self.handle, buf, n.value, C.byref(n)), "gw_profile_spans")
        return np.frombuffer(buf, dtype=np.float64)[: 3 * n.value].reshape(-1, 3).copy()

    def profile_read(self):
        """-> (ms summed over timed steps [step_kernel, obs_kernel, fear_kernel], timed steps).
        fear_kernel is nonzero only with GW_KERNEL=defer (it overlaps obs_kernel there)."""
        ms = (C.c_double * 3)()
        n = C.c_int64()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gw_profile_read(self.handle, ms, C.byref(n)), "gw_profile_read")
        return (ms[0], ms[1], ms[2]), n.value

    def positions(self) -> torch.Tensor:
        return self.state()["pos"].t().contiguous()

    def close(self):
        if not self._closed and getattr(self, "handle", None):
            self.lib.gw_destroy(self.handle)
            self._closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
