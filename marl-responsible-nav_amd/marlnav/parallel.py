"""Multi-GPU pieces: env sharding and the per-step reduction of episode statistics.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Envs are
independent units: rank r owns the contiguous global ids [offset, offset + count), and every
random draw is keyed by the global env id, so per-env trajectories are identical for any
number of ranks (tests/test_parallel.py).  The only exchange is a per-step all-reduce of the
step kernel's per-block partial sums (episode returns, completions, FeAR, crashes, apples):
a few KB per rank, latency-bound over xGMI, issued asynchronously so that the collective of
step t overlaps step t+1.
"""
from __future__ import annotations

import os

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
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


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
