"""Multi-rank batch sharding + mask all-gather with the gloo backend on CPU,
world_size 2 and 3.  The per-rank 'segmenter' is a deterministic stand-in (no GPU here);
the GPU path runs the same ShardedSegmenter with the native forward (bench.py, N>1)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from unet_mi355x.dist import ShardedSegmenter, all_gather_rows, shard_bounds


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
