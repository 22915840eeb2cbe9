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
    """Per-step gather of every rank's completed-episode returns.

    The reference appends ``scores[i]`` to ``completed_episode_scores`` for every env whose
    episode ended this step (maddpg/agent.py:229-247).  Each rank's step writes its ``[E_local]``
    f64 ``ep_return`` and u8 ``done`` (zero-copy through ``VecGridEnv.step(into=...)``).

    One rank: the step writes straight into a receive slot (no copy), and every ``window`` steps
    (and on ``completed()``) the slots are compacted on the device into a ring of the last
    ``capacity`` completed returns in the reference's order: step by step, within a step by env id.

    Several ranks (packed): only completed episodes travel.  Per step each rank appends its done
    envs' returns (env order) to a device FIFO and ONE asynchronous ``all_gather_into_tensor``
    (RCCL over xGMI) carries a fixed slot per rank: a 32-byte header (this step's count, the
    entries sent, the backlog left, an overflow flag) and up to ``cap`` returns from the FIFO's
    head -- 32 + 8 cap bytes instead of 9 bytes per env (cap = E_local / 32 by default: 16 KB at
    65,536 envs vs 576 KB).  A step with more completions than ``cap`` leaves a backlog that the
    next steps drain; every rank sees every header, so all ranks double ``cap`` at the same window
    boundary when the last window had one (a lagged host read of an already finished copy: no
    stall).  Window boundaries count pushes, not compactions: ``completed()`` / ``compact()`` may be
    called on any subset of ranks at any time (e.g. rank-0-only logging) without desynchronising
    the slot sizes.  Every ``window`` steps the receiver appends each rank's entries to a mirror FIFO and
    emits, in (step, rank, env) order, every step whose entries have all arrived -- with
    rank-major contiguous shards that is the reference's (step, global env id) order, bit for bit
    the list of the round-3 full gather (tests/test_parallel.py, tests/test_gpu_dist.py).

    The send slots are double-buffered: step t packs into buffer t & 1 while the collective of
    step t-1 still reads the other one (the stream waits on the collective of step t-2)."""

    def __init__(self, global_envs: int, rank: int, world: int, device, group=None, window: int = 64,
                 capacity: int = 1 << 20, cap: int | None = None):
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
        self.window = int(window)
        self._work = [None, None]
        self._fill = 0           # received steps not yet compacted
        self._flip = 0
        self.capacity = int(capacity)
        self.scores = torch.zeros(self.capacity + 1, dtype=torch.float64, device=self.device)  # + spare slot
        self.n_completed = torch.zeros((), dtype=torch.int64, device=self.device)  # total ever (device)
        if self.distributed:
            self._init_packed(cap)
        else:
            # packed slot: [E_max] f64 returns, then [E_max] u8 dones, padded to 8 bytes
            self.slot_bytes = 8 * self.emax + (-(-self.emax // 8)) * 8
            self._recv = torch.zeros((self.window, 1, self.slot_bytes), dtype=torch.uint8, device=self.device)
        # run the compaction once on an all-zero (nothing done) slot: loads its kernels here, not
        # inside the first timed window that compacts
        if not self.distributed:
            self._fill = 1
            self.compact()

    # ---- several ranks: the packed protocol ------------------------------------------------
    def _init_packed(self, cap):
        dev, E = self.device, self.emax
        self.cap = int(cap) if cap else max(64, -(-E // 32))
        self.cap = min(self.cap, E)
        self.fifo_cap = 2 * self.window * E + E       # a backlog the cap adaptation cannot reach
        self._ret = torch.zeros(E, dtype=torch.float64, device=dev)   # the step writes these (into())
        self._done = torch.zeros(E, dtype=torch.uint8, device=dev)
        self._fifo = torch.zeros(self.fifo_cap, dtype=torch.float64, device=dev)
        self._ctl = torch.zeros(4, dtype=torch.int64, device=dev)
        self.pend_cap = 8 * self.window
        self._mirror = torch.zeros((self.world, self.fifo_cap), dtype=torch.float64, device=dev)
        self._rst = torch.zeros(2 * self.world + 4, dtype=torch.int64, device=dev)
        self._pend = torch.zeros((self.pend_cap, self.world), dtype=torch.int32, device=dev)
        self._hip = dev.type == "cuda"
        if self._hip:
            from . import _lib
            lib = _lib.load()
            self._pack_scratch = torch.zeros(int(lib.gw_gather_pack_scratch(self.count)), dtype=torch.int32,
                                             device=dev)
            self.plan_cap = int(lib.gw_gather_unpack_plan_cap(self.window, self.world, self.pend_cap))
            self._plan = torch.zeros(self.plan_cap * 40 + 32, dtype=torch.uint8, device=dev)
            self._maxb_host = torch.zeros(2, dtype=torch.int64).pin_memory()
        else:
            self._maxb_host = torch.zeros(2, dtype=torch.int64)
        self._maxb_ev = None
        self._nwin = 0
        self._steps = 0          # pushes so far: window boundaries are multiples of `window` on every rank
        self._wmax = torch.zeros(1, dtype=torch.int64, device=dev)  # max sender backlog since the last boundary
        self._alloc_slots()

    def _alloc_slots(self):
        self.slot_bytes = 32 + 8 * self.cap
        self._send = [torch.zeros(self.slot_bytes, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self._recv = torch.zeros((self.window, self.world, self.slot_bytes), dtype=torch.uint8, device=self.device)

    def _pack(self, buf: torch.Tensor):
        if self._hip:
            import ctypes as C
            from . import _lib
            _lib.check(_lib.load().gw_gather_pack(
                self._ret.data_ptr(), self._done.data_ptr(), self.count, self.cap, self._fifo.data_ptr(),
                self.fifo_cap, self._ctl.data_ptr(), self._pack_scratch.data_ptr(), buf.data_ptr(),
                C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)), "gw_gather_pack")
            return
        # the same protocol as torch ops (CPU tensors: the gloo tests)
        new = self._ret[: self.count][self._done[: self.count] != 0]
        head, tail, ovf = (int(x) for x in self._ctl[:3])
        c = new.numel()
        if c:
            self._fifo[(tail + torch.arange(c)) % self.fifo_cap] = new
        n = min(tail - head + c, self.cap)
        payload = buf[32:].view(torch.float64)
        if n:
            payload[:n] = self._fifo[(head + torch.arange(n)) % self.fifo_cap]
        ovf = 1 if (ovf or tail - head + c > self.fifo_cap) else 0
        buf[:32].view(torch.int64).copy_(torch.tensor([c, n, tail - head + c - n, ovf]))
        self._ctl[:3] = torch.tensor([head + n, tail + c, ovf])

    def _unpack(self):
        steps = self._fill
        if self._hip:
            import ctypes as C
            from . import _lib
            _lib.check(_lib.load().gw_gather_unpack(
                self._recv.data_ptr(), steps, self.world, self.slot_bytes, self._mirror.data_ptr(), self.fifo_cap,
                self._rst.data_ptr(), self._pend.data_ptr(), self.pend_cap, self._plan.data_ptr(), self.plan_cap,
                self.scores.data_ptr(), self.capacity, self.n_completed.data_ptr(),
                C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)), "gw_gather_unpack")
            return
        W = self.world
        rst = self._rst
        recv_tot, emitted = rst[:W], rst[W:2 * W]
        maxb, bad = 0, int(rst[2 * W + 2])
        for t in range(steps):
            if int(rst[2 * W + 1] - rst[2 * W]) >= self.pend_cap:
                bad = 1
            for r in range(W):
                slot = self._recv[t, r]
                c, n, backlog, ovf = (int(x) for x in slot[:32].view(torch.int64))
                maxb, bad = max(maxb, backlog), bad | ovf
                if n:
                    idx = (int(recv_tot[r]) + torch.arange(n)) % self.fifo_cap
                    self._mirror[r, idx] = slot[32:].view(torch.float64)[:n]
                recv_tot[r] += n
                self._pend[int(rst[2 * W + 1]) % self.pend_cap, r] = c
            rst[2 * W + 1] += 1
        out = []
        while int(rst[2 * W]) < int(rst[2 * W + 1]):
            cs = self._pend[int(rst[2 * W]) % self.pend_cap]
            if not all(int(emitted[r]) + int(cs[r]) <= int(recv_tot[r]) for r in range(W)):
                break
            for r in range(W):
                c = int(cs[r])
                if c:
                    out.append(self._mirror[r, (int(emitted[r]) + torch.arange(c)) % self.fifo_cap])
                emitted[r] += c
            rst[2 * W] += 1
        rst[2 * W + 2], rst[2 * W + 3] = bad, maxb
        if out:
            vals = torch.cat(out)
            n_old = int(self.n_completed)
            keep = vals[-self.capacity:]
            dst = (n_old + len(vals) - len(keep) + torch.arange(len(keep))) % self.capacity
            self.scores[dst] = keep
            self.n_completed += len(vals)

    def overflowed(self) -> bool:
        """Whether a FIFO, mirror or pending ring ran out (the gathered list is then incomplete).
        Synchronises."""
        return self.distributed and int(self._rst[2 * self.world + 2]) != 0

    # ---- the per-step interface ------------------------------------------------------------
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
        ``done`` [E_local] (one rank: views of the receive slot; several: the packer's inputs)."""
        if self.distributed:
            return {"ep_return": self._ret[: self.count], "done": self._done[: self.count]}
        # one rank: the views of each receive slot, made once (a step's host enqueue is on the
        # critical path of short runs)
        views = self.__dict__.setdefault("_slot_views", {})
        v = views.get(self._fill)
        if v is None:
            rets, done = self._views(self._buf())
            v = views[self._fill] = {"ep_return": rets[: self.count], "done": done[: self.count]}
        return dict(v)

    def push(self, ep_return: torch.Tensor | None = None, done: torch.Tensor | None = None):
        """Gather this step's returns.  Without arguments the step wrote them through
        ``into()``; otherwise ``ep_return`` [E_local] f64 and ``done`` [E_local] u8 are copied."""
        if ep_return is not None:
            into = self.into()
            into["ep_return"].copy_(ep_return)
            into["done"].copy_(done.to(torch.uint8))
        if self.distributed:
            buf = self._buf()
            self._pack(buf)
            slot = self._recv[self._fill]
            self._work[self._flip] = dist.all_gather_into_tensor(slot.view(-1), buf, group=self.group,
                                                                 async_op=True)
            self._flip ^= 1
            self._fill += 1
            self._steps += 1
            if self._steps % self.window == 0:  # a boundary every rank reaches at the same push
                self._boundary()
            return
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
        if self.distributed:
            self._unpack()
            self._fill = 0
            # the backlog maximum over every unpack since the last boundary: the same steps' headers
            # on every rank, however a rank split them into compactions (completed() mid-window)
            w = 2 * self.world + 3
            torch.maximum(self._wmax, self._rst[w:w + 1], out=self._wmax)
            return
        if self._recv.is_cuda:
            self._compact_hip()
            return
        self._compact_torch()

    def drain(self, max_steps: int = 1 << 20) -> int:
        """COLLECTIVE (every rank calls it at the same point): gather steps with no new completions
        until no rank has a backlog, so that ``completed()`` holds every episode that ended, even in
        a run that stopped right after a completion burst larger than ``cap``.  The loop condition is
        read from the gathered headers, which every rank holds alike.  Returns the steps added (0
        with one rank)."""
        if not self.distributed:
            return 0
        added = 0
        while added < max_steps:
            buf = self._buf()
            self._done.zero_()   # this pseudo-step completes nothing; the step's outputs were packed
            self._pack(buf)
            slot = self._recv[self._fill]
            dist.all_gather_into_tensor(slot.view(-1), buf, group=self.group)
            backlog = int(slot[:, :32].view(torch.int64)[:, 2].max())  # header: count, sent, backlog, ovf
            self._flip ^= 1
            self._fill += 1
            self._steps += 1
            added += 1
            if self._steps % self.window == 0:
                self._boundary()
            if backlog == 0:
                break
        self.compact()
        return added

    def _boundary(self):
        """Every ``window`` pushes (the same pushes on every rank, whatever compact() / completed()
        calls a rank made in between): fold the received steps in, copy the window's maximum sender
        backlog to the host (read one window later: no stall) and adapt ``cap`` from the window
        before.  The decision depends only on gathered headers and the push count, so every rank
        resizes its slots at the same step."""
        self.compact()
        slot = self._nwin % 2
        self._maxb_host[slot:slot + 1].copy_(self._wmax, non_blocking=self._hip)
        self._wmax.zero_()
        prev_ev = None
        if self._hip:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            prev_ev, self._maxb_ev = self._maxb_ev, ev
        self._nwin += 1
        if self._nwin >= 2:
            self._adapt_from(prev_ev)

    def _adapt_from(self, ev):
        """Grow ``cap`` (x2, up to the shard) when the window before this one left a backlog on any
        rank.  Every rank reads the same gathered headers, so all ranks decide alike; the value was
        copied a whole window ago, so the wait is normally on a long finished event."""
        if ev is not None:
            ev.synchronize()
        prev = int(self._maxb_host[(self._nwin - 2) % 2])
        if prev > 0 and self.cap < self.emax:
            self.cap = min(2 * self.cap, self.emax)
            self._alloc_slots()

    def _compact_hip(self):
        """gw_return_compact (include/rollout_ops.h): count + scatter, two launches."""
        import ctypes as C
        from . import _lib
        lib = _lib.load()
        world = self._recv.shape[1]  # 1 here; the kernel takes any rank count (its tests use several)
        need = int(lib.gw_return_compact_scratch(self._fill, world, self.emax))
        if getattr(self, "_scratch", None) is None or self._scratch.numel() < need:
            self._scratch = torch.zeros(max(need, 2 + (self.window * self.emax + 4095) // 4096),
                                        dtype=torch.int32, device=self.device)
        _lib.check(lib.gw_return_compact(self._recv.data_ptr(), self._fill, world, self.emax, self.slot_bytes,
                                         self.scores.data_ptr(), self.capacity, self.n_completed.data_ptr(),
                                         self._scratch.data_ptr(),
                                         C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "gw_return_compact")
        self._fill = 0

    def _compact_torch(self):
        """The same compaction as torch ops (CPU tensors: single-process tests)."""
        block = self._recv[: self._fill]                               # [T, 1, slot]
        rets = block.view(torch.float64)[:, :, : self.emax]            # [T, 1, E_max] (slot_bytes % 8 == 0)
        done = block[:, :, 8 * self.emax: 9 * self.emax] != 0
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
        if self.overflowed():
            raise RuntimeError("ReturnGather: a FIFO / mirror / pending ring overflowed (completions per step far "
                               "above cap for two windows); raise cap")
        n = int(self.n_completed.item())
        m = min(n, self.capacity) if last is None else min(n, self.capacity, int(last))
        if m == 0:
            return np.zeros(0, np.float64)
        start = (n - m) % self.capacity
        idx = (torch.arange(m, device=self.device) + start) % self.capacity
        return self.scores[idx].cpu().numpy()
