"""bench.py's launcher, scaling modes and per-launch accounting, on CPU (no GPU here).

The launcher runs with the CPU stand-in forward (``--standin``: gloo, a deterministic function of
each image into the bit-packed mask shape) through the same sharding, preallocated all-gather and
timing code as the GPU run, in both launch modes the driver may use: ``python bench.py --gpus N``
(bench.py spawns its N ranks itself) and ``torch.distributed.run`` (WORLD_SIZE set)."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
SMALL = ["--standin", "--size", "32", "--steps", "3", "--warmup", "1"]


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _run(cmd, env=None, timeout=180):
    p = subprocess.run(cmd, cwd=REPO, env=env or _env(), capture_output=True, text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p, lines


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_self_spawn_weak_scaling():
    p, lines = _run([sys.executable, BENCH, "--gpus", "2", "--batch", "4"] + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout                 # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["config"]["global_batch"] == 8 and out["config"]["per_gpu_batch"] == 4
    assert out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["config"]["exchange"] == "all_gather_into_tensor"


def test_self_spawn_strong_scaling_ragged():
    p, lines = _run([sys.executable, BENCH, "--gpus", "3", "--global-batch", "10"] + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["scaling"] == "strong"
    assert out["config"]["global_batch"] == 10 and out["config"]["per_gpu_batch"] == 4   # 4 + 3 + 3


def test_strong_legs_chunked_two_ranks():
    """A strong-scaling leg whose shard is larger than the workspace chunk (global 10 over 2 ranks =
    5 images per rank, chunk = --batch 2) runs as 3 chunked forwards + the one all-gather, at
    world 2 -- the path the strong_1024 leg takes on 1 and 2 GPUs."""
    p, lines = _run([sys.executable, BENCH, "--gpus", "2", "--batch", "2", "--strong-global", "10"] + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(lines[0])
    (leg,) = out["strong_scaling"]
    assert leg["global_batch"] == 10 and leg["per_rank_batch"] == [5, 5] and leg["value"] > 0


def test_torchrun_launch():
    p, lines = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                     "--master-addr", "127.0.0.1", "--master-port", str(_port()), BENCH, "--gpus", "2",
                     "--batch", "2"] + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 4


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_world_eight_ragged_strong_legs(launcher, tmp_path):
    """The driver's N = 8 launch, both ways (bench.py spawning its 8 ranks / torch.distributed.run), with
    the strong-scaling legs of north_star (global 256: 32 per rank) and config 4 (global 1024, chunked
    forwards of --batch images) plus a ragged global batch (1021 = 5 x 128 + 3 x 127): the line reports
    the MAX-over-ranks compute time beside the all-gather's, and the ragged shard sizes."""
    detail = tmp_path / "d.json"
    args = [BENCH, "--gpus", "8", "--batch", "32", "--strong-global", "256", "1024", "1021",
            "--detail-out", str(detail), "--standin", "--size", "16", "--steps", "2", "--warmup", "1"]
    if launcher == "self":
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    p, lines = _run(cmd, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["config"]["global_batch"] == 256 and out["config"]["per_gpu_batch"] == 32
    assert out["allgather_ms"] is not None and out["compute_ms"] is not None
    assert 0 < out["compute_ms_min"] <= out["compute_ms"] < out["ms_per_step"] + 1e-6
    legs = {leg["global_batch"]: leg for leg in out["strong_scaling"]}
    assert legs[256]["per_rank_batch"] == [32] * 8
    assert legs[1024]["per_rank_batch"] == [128] * 8
    assert legs[1021]["per_rank_batch"] == [128] * 5 + [127] * 3
    assert all(leg["value"] > 0 for leg in legs.values())
    rec = json.loads(detail.read_text())
    assert len(rec["detail"]["compute_ms"]) == 2 and len(rec["detail"]["allgather_ms"]) == 2


def test_world_size_mismatch_fails_instead_of_benchmarking_one_gpu():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    p, lines = _run([sys.executable, BENCH, "--gpus", "2", "--batch", "2"] + SMALL, env=env)
    assert p.returncode == 2 and not lines
    assert "WORLD_SIZE=1" in p.stderr


def test_spawned_rank_failure_propagates():
    # rank 1 exits before its first collective; rank 0 would wait in the barrier forever: the
    # launcher stops it and reports the failure
    env = _env()
    env["BENCH_FAIL_RANK"] = "1"
    p, lines = _run([sys.executable, BENCH, "--gpus", "2", "--batch", "2"] + SMALL, env=env, timeout=120)
    assert p.returncode == 3 and not lines


def test_launch_table_credits_each_kernel_with_its_own_work():
    sys.path.insert(0, REPO)
    import bench
    n, s, c, e = 256, 512, 3, 2
    labels = ["x_to_px4_kernel<_Float16>"] + [f"k{i}" for i in range(1, 22)]
    labels[19] = ""   # up1 fused into conv2.3
    rows = bench.launch_table(labels, n, s, s, c, e)
    total = sum(bench.launch_flops(en, n, s, s, c) for en in bench.LAUNCHES)
    assert sum(r[2] for r in rows) == pytest.approx(total)
    assert rows[0][2] == 0 and rows[0][3] == n * s * s * (c * 4 + 4 * e)     # the cast: 3 + 2 MB per image
    first = bench.launch_flops(bench.LAUNCHES[0], n, s, s, c)
    assert rows[1][2] == pytest.approx(first + bench.launch_flops(bench.LAUNCHES[1], n, s, s, c))
    assert rows[19][2] == 0 and rows[19][1] == "k18" and not rows[19][4]
    up1 = bench.launch_flops(bench.LAUNCHES[19], n, s, s, c)
    assert rows[18][2] == pytest.approx(bench.launch_flops(bench.LAUNCHES[18], n, s, s, c) + up1)
    # the cast ran 0.328 ms in r2p: its credited bytes must be a possible HBM rate (round 2 credited it
    # with down1.0's 9.4 GB = 28.7 TB/s)
    assert rows[0][3] / 0.328e-3 < 8e12
    # the fused conv2.3 + up1 neither writes nor re-reads x2 (128 ch at 256^2)
    x2 = n * (s // 2) ** 2 * 128 * e
    assert rows[18][3] == (bench.launch_bytes(bench.LAUNCHES[18], n, s, s, c, e) +
                           bench.launch_bytes(bench.LAUNCHES[19], n, s, s, c, e) - 2 * x2)


def test_pmc_summary_labels_mangled_and_demangled_names():
    """rocprofv3 demangles some kernel names (the fp32 kernels) and leaves the 16-bit ones mangled:
    both must map to bench.py's kernel labels, or the roofline's traffic comes out as 0."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from pmc_summary import label_of
    assert label_of("void unet::conv3x3_halo_kernel<float, 1, 4, 8, 2, 3, 0>(unet::IgemmArgs)") == \
        "conv3x3_halo_kernel<float, 1, 4, 8, 2, 3, 0>"
    assert label_of("_ZN4unet20conv3x3_ring8_kernelIDF16bLi8ELi3ELi0ELi3ELi0EDF16bDF16bLi0ELi0EEEvNS_9IgemmArgsE") == \
        "conv3x3_ring8_kernel<__bf16, 8, 3, 0, 3, 0, __bf16, __bf16, 0, 0>"


def test_dist_mode_at_world_one_runs_the_exchange(tmp_path):
    """--dist at world size 1: the process group is initialised (gloo here, nccl on a GPU) and the
    step runs the N > 1 exchange -- all_gather_into_tensor into a separate receive buffer, barriers
    and the MAX all-reduce -- so the multi-GPU code path runs on a one-GPU box."""
    detail = tmp_path / "detail.json"
    p, lines = _run([sys.executable, BENCH, "--gpus", "1", "--dist", "--batch", "4", "--detail-out", str(detail)]
                    + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["exchange"] == "all_gather_into_tensor"
    assert out["config"]["parallelism"] == "dp1"
    rec = json.loads(detail.read_text())
    assert rec["summary"]["value"] == out["value"] and len(rec["detail"]["host_step_ms"]) == 3
    # without --dist nothing is exchanged at world 1
    p, lines = _run([sys.executable, BENCH, "--gpus", "1", "--batch", "4", "--detail-out", ""] + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    assert json.loads(lines[0])["config"]["exchange"] is None


def test_summary_line_is_compact():
    """The driver keeps the last 8 KB of stdout: the one JSON line must fit with room to spare; the
    per-kernel tables and per-step times go to the detail record (stderr and --detail-out)."""
    p, lines = _run([sys.executable, BENCH, "--gpus", "2", "--batch", "2", "--detail-out", ""] + SMALL)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines[0]) < 4096
    out = json.loads(lines[0])
    assert "kernels" not in out and "step_ms" not in out
    assert "bench_detail " in p.stderr
