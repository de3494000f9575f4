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


def all_gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Gather the per-rank shards (dim 0, sizes per shard_bounds) into the full batch.

    Shards are padded to the largest shard so one all_gather_into_tensor covers ragged
    batches; the padding is dropped on return.  Order = rank order = original batch order.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(n_total, rank, world)
    if local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: local shard has {local.shape[0]} rows, expected {hi - lo}")
    cap = shard_bounds(n_total, 0, world)[1]          # largest shard (rank 0)
    if local.shape[0] < cap:
        pad = torch.zeros((cap - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send = torch.cat([local, pad], 0)
    else:
        send = local.contiguous()
    out = torch.empty((world * cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, send, group=group)   # RCCL over xGMI with "nccl"; gloo on CPU
    if n_total % world == 0:
        return out
    keep = []
    for r in range(world):
        a, b = shard_bounds(n_total, r, world)
        keep.append(out[r * cap: r * cap + (b - a)])
    return torch.cat(keep, 0)


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


def timed_steps(step, steps: int, warmup: int, sync=None, device=None, group=None) -> tuple[float, list]:
    """The bench contract's timing loop (bench.py): ``warmup`` untimed steps, then exactly
    ``steps`` timed steps bracketed by a barrier + ``sync()`` on both sides; returns the
    elapsed seconds as the MAX over ranks (one all-reduce on ``device``: the GPU with "nccl",
    the CPU with gloo) and the per-step host times of this rank.  ``step`` runs one step (for
    N > 1 its forward and the mask all-gather)."""
    sync = sync or (lambda: None)
    distributed = dist.is_initialized() and dist.get_world_size(group) > 1
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


def sharded_mask_step(segment_fn, x_local: torch.Tensor, masks_local: torch.Tensor, n_total: int, group=None):
    """One data-parallel step of bench.py at N > 1: this rank's forward of its shard into its
    (bit-packed) mask buffer, then the one exchange step -- the all-gather of every rank's masks.
    Returns the gathered masks [n_total, ...] in global batch order."""
    segment_fn(x_local, masks_local)
    return all_gather_rows(masks_local, n_total, group)
