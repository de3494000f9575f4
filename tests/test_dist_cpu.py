"""Multi-rank batch sharding + mask all-gather with the gloo backend on CPU,
world_size 2 and 3.  The collective is the same call the bench's RCCL path makes
(all_gather_into_tensor; gloo implements it on CPU), and the bench's N>1 step and timing loop
(unet_mi355x.dist.sharded_mask_step / timed_steps: bench.py's step calls sharded_mask_step whenever a
shard fits one forward, and runs the same forward per chunk + the same gather otherwise, which
tests/test_bench_cpu.py::test_strong_legs_chunked_two_ranks covers) run here with a
deterministic CPU stand-in for the per-rank forward (no GPU here)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import time

from unet_mi355x.dist import MaskGather, ShardedSegmenter, all_gather_rows, shard_bounds, sharded_mask_step, timed_steps


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_masks(x):
    # bit-packed-mask shaped output that depends on each image only
    return (x.sum(dim=(1, 2, 3), keepdim=True).abs().floor().to(torch.uint8) + torch.arange(8, dtype=torch.uint8)
            ).expand(-1, 3, 4, 8).contiguous()


def fake_boxes(x):
    # unet_forward_boxes-shaped output: int32 [n, 3, 4], -1s for "empty" fields
    v = (x.sum(dim=(1, 2, 3)).abs() * 10).floor().to(torch.int32)
    b = torch.stack([v, v + 1, v + 2, v + 3], -1).unsqueeze(1).repeat(1, 3, 1)
    b[v % 3 == 0, 1] = -1
    return b.contiguous()


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        x = torch.randn(n_total, 3, 16, 16)
        seg = ShardedSegmenter(fake_masks)
        got = seg(x)
        ref = fake_masks(x)
        lo, hi = shard_bounds(n_total, rank, world)
        got2 = seg(x[lo:hi], n_total=n_total, already_local=True)
        boxes = ShardedSegmenter(fake_boxes)(x)     # the 48-byte-per-image gather of §8f
        ok2 = bool(torch.equal(got2, ref)) and bool(torch.equal(boxes, fake_boxes(x)))
        q.put((rank, bool(torch.equal(got, ref)), ok2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 8), (2, 7), (3, 10)])
def test_sharded_gather_equals_single_process(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r for r, _, _ in res) == list(range(world))
    assert all(a and b for _, a, b in res), res


def test_shard_bounds_cover_batch():
    for n in (1, 7, 256, 1000):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def _bench_worker(rank, world, port, per_rank, q):
    """bench.py's N>1 step: each rank holds its own per-GPU batch (weak scaling), forwards it
    into its bit-packed mask buffer and all-gathers; timing = max over ranks."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        x_global = torch.randn(world * per_rank, 3, 16, 16)
        x_local = x_global[rank * per_rank:(rank + 1) * per_rank].contiguous()
        gather = MaskGather(world * per_rank, (3, 4, 8), torch.uint8, "cpu")
        out_ptr = gather.out.data_ptr()
        calls = []

        def segment(xl, ml):       # stand-in for handle.forward(x, None, masks, MASK_BITS, stream)
            ml.copy_(fake_masks(xl))
            calls.append(xl.shape[0])

        gathered = []

        def step():
            time.sleep(0.02 * (rank + 1))        # ranks finish at different times
            gathered.append(sharded_mask_step(segment, x_local, gather).clone())

        elapsed, per_step = timed_steps(step, steps=3, warmup=1)
        ok = all(torch.equal(g, fake_masks(x_global)) for g in gathered) and len(gathered) == 4
        ok = ok and gather.out.data_ptr() == out_ptr     # the exchange reuses its preallocated buffers
        # the reported time is the slowest rank's: >= 3 steps of the last rank's 0.02*world s
        q.put((rank, ok, elapsed >= 3 * 0.02 * world, len(per_step) == 3 and calls == [per_rank] * 4))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank", [(2, 4), (3, 2)])
def test_bench_step_and_timing_under_gloo(world, per_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in res) == list(range(world))
    assert all(all(r[1:]) for r in res), res
