"""Batch data-parallel inference across the GPUs of one node.

Images are independent (eval-mode BatchNorm, no cross-batch coupling), so a global batch is
split contiguously over ranks -- one process per GPU, rank r gets
[r*N/P, (r+1)*N/P) -- every rank runs the native forward on its shard with a full weight
replica, and the only exchange step is ONE all-gather of the (bit-packed) masks.  With the
"nccl" backend that collective is RCCL over xGMI; with "gloo" (CPU tests) it is the same
code path.  The reference has no parallelism at all (single device, inference.py:9).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of rank; the first n_total % world ranks get one extra."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class MaskGather:
    """The one exchange step with its buffers allocated once: every rank writes its shard into
    ``local`` (the first hi - lo rows of a send buffer padded to the largest shard, padding rows
    zero), and ``__call__`` all-gathers the send buffers into ``out`` ([world x cap] rows, rank r's
    shard at rows [r cap, r cap + its size)).  ``rows()`` drops the padding (a copy, outside any
    timed step).  With "nccl" the collective is RCCL over xGMI; with gloo the same call on CPU.

    ``collective``: None = run the all-gather only when world > 1; True = run it at every world size
    (bench.py --dist: the N > 1 code path -- RCCL all_gather_into_tensor into a separate receive
    buffer -- exercised on a one-GPU box)."""

    def __init__(self, n_total: int, row_shape, dtype, device, group=None, rank=None, world=None,
                 collective=None):
        self.group = group
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        self.collective = self.world > 1 if collective is None else bool(collective)
        if self.collective and not dist.is_initialized():
            raise RuntimeError("MaskGather(collective=True) needs an initialised process group")
        self.n_total = n_total
        lo, hi = shard_bounds(n_total, self.rank, self.world)
        self.cap = shard_bounds(n_total, 0, self.world)[1]          # largest shard (rank 0)
        self.send = torch.zeros((self.cap,) + tuple(row_shape), dtype=dtype, device=device)
        self.local = self.send[:hi - lo]
        self.out = self.send if not self.collective else \
            torch.empty((self.world * self.cap,) + tuple(row_shape), dtype=dtype, device=device)

    def __call__(self) -> torch.Tensor:
        if self.collective:
            dist.all_gather_into_tensor(self.out, self.send, group=self.group)
        return self.out

    def rows(self) -> torch.Tensor:
        """The gathered shards in global batch order without the padding rows."""
        if self.n_total % self.world == 0:
            return self.out
        keep = []
        for r in range(self.world):
            a, b = shard_bounds(self.n_total, r, self.world)
            keep.append(self.out[r * self.cap: r * self.cap + (b - a)])
        return torch.cat(keep, 0)


def all_gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Gather the per-rank shards (dim 0, sizes per shard_bounds) into the full batch, in rank
    order = original batch order (one-shot form of MaskGather: allocates its buffers per call)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(n_total, rank, world)
    if local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: local shard has {local.shape[0]} rows, expected {hi - lo}")
    g = MaskGather(n_total, tuple(local.shape[1:]), local.dtype, local.device, group, rank, world)
    g.local.copy_(local)
    g()
    return g.rows()


class ShardedSegmenter:
    """Runs ``segment_fn`` (e.g. ``lambda x: model.forward_masks(x, packed=True)``) on this
    rank's shard of a global batch and all-gathers the masks to every rank."""

    def __init__(self, segment_fn, group=None):
        self.segment_fn = segment_fn
        self.group = group

    def __call__(self, x_global_or_local: torch.Tensor, n_total: int | None = None,
                 already_local: bool = False) -> torch.Tensor:
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        if already_local:
            if n_total is None:
                raise ValueError("n_total is required with already_local=True")
            local = x_global_or_local
        else:
            n_total = x_global_or_local.shape[0]
            lo, hi = shard_bounds(n_total, rank, world)
            local = x_global_or_local[lo:hi]
        masks = self.segment_fn(local)
        return all_gather_rows(masks, n_total, self.group)


def timed_steps(step, steps: int, warmup: int, sync=None, device=None, group=None,
                collective=None) -> tuple[float, list]:
    """The bench contract's timing loop (bench.py): ``warmup`` untimed steps, then exactly
    ``steps`` timed steps bracketed by a barrier + ``sync()`` on both sides; returns the
    elapsed seconds as the MAX over ranks (one all-reduce on ``device``: the GPU with "nccl",
    the CPU with gloo) and the per-step host times of this rank.  ``step`` runs one step (for
    N > 1 its forward and the mask all-gather).  ``collective=True`` runs the barriers and the
    all-reduce at world size 1 too (bench.py --dist)."""
    sync = sync or (lambda: None)
    distributed = dist.is_initialized() and (dist.get_world_size(group) > 1 or bool(collective))
    for _ in range(warmup):
        step()
    if distributed:
        dist.barrier(group=group)
    sync()
    marks = [time.perf_counter()]
    for _ in range(steps):
        step()
        marks.append(time.perf_counter())
    sync()
    if distributed:
        dist.barrier(group=group)
    elapsed = time.perf_counter() - marks[0]
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        elapsed = float(t.item())
    return elapsed, [b - a for a, b in zip(marks, marks[1:])]


def sharded_mask_step(segment_fn, x_local: torch.Tensor, gather: MaskGather):
    """One data-parallel step of bench.py at N > 1: this rank's forward of its shard into its slot of
    the preallocated send buffer (``gather.local``, bit-packed masks), then the one exchange step --
    the all-gather of every rank's masks into ``gather.out``.  Allocates nothing."""
    segment_fn(x_local, gather.local)
    return gather()
