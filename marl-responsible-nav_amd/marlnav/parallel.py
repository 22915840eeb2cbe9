"""Multi-GPU pieces: env sharding, the per-step gather of episode returns, replicated weights.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Envs are
independent units: rank r owns the contiguous global ids [offset, offset + count), and every
random draw is keyed by the global env id, so per-env trajectories are identical for any
number of ranks (tests/test_parallel.py).  The only per-step exchange is the all-gather of
every env's episode return and done flag (ReturnGather: 9 bytes per env, asynchronous, SURVEY.md
§8e).  Episode statistics are summed by the step kernels into a per-rank running total and
all-reduced only when read (Rollout.totals); StatsReducer remains for callers that want a
per-step reduction of partial sums.  Weights are replicated by broadcast (broadcast_module,
MADDPG.broadcast_parameters) and kept equal by the learner's gradient all-reduce.
"""
from __future__ import annotations

import os

import numpy as np

import torch
import torch.distributed as dist


def shard(global_envs: int, rank: int, world: int):
    """Contiguous env range of `rank`: (offset, count); sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(int(global_envs), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun); returns
    (rank, world, local_rank).  Single process -> (0, 1, 0) without a process group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:  # MARLNAV_DIST_BACKEND=gloo rehearses several ranks on one GPU
            backend = os.environ.get("MARLNAV_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0, group=None):
    """Replicate a module's parameters and buffers from rank ``src`` (one broadcast of their
    coalesced values), e.g. actors that act without a learner (actor weights are
    broadcast once at start).  No-op without a process group of more than one rank."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
    ts = [t.detach() for t in list(module.parameters()) + list(module.buffers())]
    if not ts:
        return
    buf = _flatten_dense_tensors(ts)
    dist.broadcast(buf, src, group=group)
    for t, v in zip(ts, _unflatten_dense_tensors(buf, ts)):
        t.copy_(v)
    if hasattr(module, "mark_updated"):
        module.mark_updated()


class StatsReducer:
    """Asynchronous, double-buffered all-reduce of [rows, F] partial-sum tensors.

    push(x) enqueues the reduction of x's rows (summed over rows first, so the message is F
    doubles) and returns immediately; the previous step's collective is waited for and folded
    into `totals`.  With world size 1 (or no group) it reduces locally."""

    def __init__(self, n_fields: int, device, group=None):
        self.group = group
        self.totals = torch.zeros(n_fields, dtype=torch.float64, device=device)
        self._pending = None
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self._bufs = [torch.zeros(n_fields, dtype=torch.float64, device=device) for _ in range(2)]
        self._flip = 0

    def push(self, partials: torch.Tensor, counter: torch.Tensor | None = None):
        """Fold one step's [rows, F] partial sums in; ``counter`` (int64 device scalar, e.g. the
        replay ring's step count) is incremented in the same launch.  On the GPU this is ONE
        gw_rollout_tick launch (include/rollout_ops.h); CPU tensors (gloo tests) use torch ops."""
        self._drain()
        if partials.dim() == 1:
            partials = partials.unsqueeze(0)
        if partials.is_cuda:
            import ctypes as C
            from . import _lib
            lib = _lib.load()
            buf = self._bufs[self._flip] if self.distributed else None
            self._flip ^= 1
            assert partials.dtype == torch.float64 and partials.is_contiguous()
            assert counter is None or (counter.dtype == torch.int64 and counter.is_cuda)
            _lib.check(lib.gw_rollout_tick(partials.data_ptr(), partials.shape[0], partials.shape[1],
                                           buf.data_ptr() if buf is not None else None,
                                           None if self.distributed else self.totals.data_ptr(),
                                           counter.data_ptr() if counter is not None else None,
                                           C.c_void_p(torch.cuda.current_stream(partials.device).cuda_stream)),
                       "gw_rollout_tick")
            local = buf
        else:
            local = partials.sum(0)
            if counter is not None:
                counter.add_(1)
            if not self.distributed:
                self.totals += local
        if self.distributed:
            work = dist.all_reduce(local, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._pending = (work, local)

    def _drain(self):
        if self._pending is not None:
            work, buf = self._pending
            work.wait()
            self.totals += buf
            self._pending = None

    def result(self) -> torch.Tensor:
        self._drain()
        return self.totals


class ReturnGather:
    """Per-step all-gather of every env's completed-episode return.

    The reference appends ``scores[i]`` to ``completed_episode_scores`` for every env whose
    episode ended this step (maddpg/agent.py:229-247).  Here each rank's step writes its
    ``[E_local]`` f64 ``ep_return`` and u8 ``done`` straight into one packed send buffer
    (zero-copy through ``VecGridEnv.step(into=...)``; shards shorter than the longest are padded
    with done = 0), and ONE asynchronous ``all_gather_into_tensor`` (RCCL over xGMI on the GPU)
    delivers ``[world][E_max]`` returns + dones to every rank: 9 bytes per env per step.

    Received steps accumulate in a device ring of ``window`` slots; every ``window`` steps (and
    on ``completed()``) they are compacted on the device, with no host synchronisation, into a
    ring of the last ``capacity`` completed returns in the reference's order: step by step, and
    within a step by global env id.  ``completed()`` returns them to the host (it synchronises).

    Double-buffered: step t writes send buffer t & 1 while the collective of step t-1 still
    reads the other one; the stream waits on the collective of step t-2 before its buffer is
    overwritten (a device-side wait, not a host one).  With one rank the step writes the
    receive slot directly."""

    def __init__(self, global_envs: int, rank: int, world: int, device, group=None, window: int = 64,
                 capacity: int = 1 << 20):
        self.group = group
        self.rank, self.world = int(rank), int(world)
        self.G = int(global_envs)
        self.offset, self.count = shard(self.G, self.rank, self.world)
        self.emax = -(-self.G // self.world)
        self.device = torch.device(device)
        self.distributed = (self.world > 1 and dist.is_available() and dist.is_initialized()
                            and dist.get_world_size(group) > 1)
        if self.world > 1 and not self.distributed:
            raise RuntimeError("ReturnGather: world > 1 needs an initialised process group")
        # packed slot: [E_max] f64 returns, then [E_max] u8 dones, padded to 8 bytes
        self.slot_bytes = 8 * self.emax + (-(-self.emax // 8)) * 8
        self._send = [torch.zeros(self.slot_bytes, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self._work = [None, None]
        self.window = int(window)
        self._recv = torch.zeros((self.window, self.world, self.slot_bytes), dtype=torch.uint8, device=self.device)
        self._fill = 0           # received steps not yet compacted
        self._flip = 0
        self.capacity = int(capacity)
        self.scores = torch.zeros(self.capacity + 1, dtype=torch.float64, device=self.device)  # + spare slot
        self.n_completed = torch.zeros((), dtype=torch.int64, device=self.device)  # total ever (device)
        # run the compaction once on an all-zero (no episode done) slot: loads its kernels here,
        # not inside the first timed window that compacts
        self._fill = 1
        self.compact()

    def _views(self, buf: torch.Tensor):
        rets = buf[: 8 * self.emax].view(torch.float64)
        done = buf[8 * self.emax: 9 * self.emax]
        return rets, done

    def _buf(self) -> torch.Tensor:
        """This step's send buffer; with one rank the receive slot itself (no copy at all)."""
        if not self.distributed:
            return self._recv[self._fill, 0]
        w = self._work[self._flip]
        if w is not None:   # the collective that last read this buffer (step t-2)
            w.wait()
            self._work[self._flip] = None
        return self._send[self._flip]

    def into(self) -> dict:
        """Output buffers for this rank's next ``VecGridEnv.step(into=...)``: ``ep_return`` and
        ``done`` views of the current send buffer (its first E_local entries)."""
        rets, done = self._views(self._buf())
        return {"ep_return": rets[: self.count], "done": done[: self.count]}

    def push(self, ep_return: torch.Tensor | None = None, done: torch.Tensor | None = None):
        """Gather this step's returns.  Without arguments the step wrote them through
        ``into()``; otherwise ``ep_return`` [E_local] f64 and ``done`` [E_local] u8 are copied."""
        buf = self._buf()
        if ep_return is not None:
            rets, dn = self._views(buf)
            rets[: self.count].copy_(ep_return)
            dn[: self.count].copy_(done.to(torch.uint8))
        if self.distributed:
            slot = self._recv[self._fill]
            self._work[self._flip] = dist.all_gather_into_tensor(slot.view(-1), buf, group=self.group,
                                                                 async_op=True)
            self._flip ^= 1
        self._fill += 1
        if self._fill == self.window:
            self.compact()

    def compact(self):
        """Fold the received steps into the score ring, on the device (no host sync)."""
        if self._fill == 0:
            return
        for w in self._work:   # the slots written by collectives still in flight
            if w is not None:
                w.wait()
        self._work = [None, None]
        if self._recv.is_cuda:
            self._compact_hip()
            return
        self._compact_torch()

    def _compact_hip(self):
        """gw_return_compact (include/rollout_ops.h): count + scatter, two launches."""
        import ctypes as C
        from . import _lib
        lib = _lib.load()
        need = int(lib.gw_return_compact_scratch(self._fill, self.world, self.emax))
        if getattr(self, "_scratch", None) is None or self._scratch.numel() < need:
            self._scratch = torch.zeros(max(need, 2 + (self.window * self.world * self.emax + 4095) // 4096),
                                        dtype=torch.int32, device=self.device)
        _lib.check(lib.gw_return_compact(self._recv.data_ptr(), self._fill, self.world, self.emax, self.slot_bytes,
                                         self.scores.data_ptr(), self.capacity, self.n_completed.data_ptr(),
                                         self._scratch.data_ptr(),
                                         C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "gw_return_compact")
        self._fill = 0

    def _compact_torch(self):
        """The same compaction as torch ops (CPU tensors: the gloo tests; the GPU test's reference)."""
        block = self._recv[: self._fill]                               # [T, world, slot]
        rets = block.view(torch.float64)[:, :, : self.emax]            # [T, world, E_max] (slot_bytes % 8 == 0)
        done = block[:, :, 8 * self.emax: 9 * self.emax] != 0
        # order: step, then global env id (rank-major contiguous shards)
        rets, done = rets.reshape(-1), done.reshape(-1)
        pos = torch.cumsum(done, 0, dtype=torch.int64)
        # only the last `capacity` completions can survive; every other element (not done, or
        # overwritten within this block) is sent to the spare slot at index `capacity`, so the
        # scatter has a static shape (no host synchronisation) and no two kept writes collide
        keep = done & (pos > pos[-1] - self.capacity)
        dst = torch.where(keep, (self.n_completed + pos - 1) % self.capacity, self.capacity)
        self.scores.index_put_((dst,), rets)
        self.n_completed += pos[-1]
        self._fill = 0

    def completed(self, last: int | None = None) -> np.ndarray:
        """The completed-episode returns gathered so far (the last ``capacity`` at most), oldest
        first, on the host; ``last`` keeps only the most recent ones (the reference averages
        ``[-100:]`` style windows).  Synchronises."""
        self.compact()
        n = int(self.n_completed.item())
        m = min(n, self.capacity) if last is None else min(n, self.capacity, int(last))
        if m == 0:
            return np.zeros(0, np.float64)
        start = (n - m) % self.capacity
        idx = (torch.arange(m, device=self.device) + start) % self.capacity
        return self.scores[idx].cpu().numpy()
