#!/usr/bin/env python
"""bench.py -- invoice masks/sec of the MI355X UNet forward path (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic invoice pages resident in
HBM: UNet(3,3) forward at 512x512 (unet_model.py:55-86) with the fused sigmoid +
per-field threshold (inference.py:72-79) producing bit-packed masks, plus -- for N>1 --
the RCCL all-gather of the masks over xGMI into a preallocated buffer.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256] [--global-batch G] [--dtype mixed]
    torchrun --nproc-per-node N bench.py --gpus N ...      (the driver does this for N>1)

Launch: under torchrun (WORLD_SIZE set) every process is one rank; WORLD_SIZE must equal --gpus
(exit 2 otherwise).  Without WORLD_SIZE and --gpus N > 1 the script spawns its own N rank
processes (127.0.0.1 rendezvous) before any GPU call and exits with the worst rank's code.

Scaling: by default every GPU holds --batch images per step (weak scaling, the headline `value`);
--global-batch G splits G images over the ranks instead (strong scaling).  The same run also
times the strong-scaling shapes of BASELINE's multi-GPU configurations -- global batch 256
(north_star's "1 -> 8 GPUs at batch 256": 32 images per rank at N = 8) and 1024 (config 4: 128
per rank) -- as `strong_scaling`.

Rank 0 prints ONE JSON line.  Extra fields: roofline (dominant kernel, HIP-event timed inside
this run), cpu_baseline (the oracle on this host's cores, bounded sample), fp32 (BASELINE
config 2: batch 32, 512^2, the drop-in's default precision, against the 157.3 TF fp32 MFMA
peak), cfg5 (BASELINE config 5 per GPU: 1024^2, fp16, batch 64), latency_bs1 (the drop-in run_unet
and the batch-1 forward at the drop-in default fp32 and at the bench plan, with a per-layer
breakdown), kernels (per-instantiation time breakdown).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import re
import socket
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from unet_mi355x import dist as udist  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402

METRIC = "invoice masks/sec at 512x512 bs256, 1/2/4/8 MI355X; IoU vs CPU ref"
# dense MFMA peaks (MI355X_MICROARCH.md).  "fp32" runs every product as 6 bf16 MFMA products (three bf16 terms per
# operand), so its ceiling in fp32 FLOPs is the bf16 peak / 6; "fp32_exact" runs v_mfma_f32_16x16x4_f32.
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "mixed": 2500.0, "fp32": 2500.0 / 6, "fp32_exact": 157.3}
HBM_PEAK_GBS = 8000.0
HEAD16 = ("1x1 head on 16-bit MFMA operands (conv1.3's ReLU outputs and the out_conv weights rounded to the "
          "layer's type), fp32 accumulation and fp32 bias")
PLAN = {"mixed": "bf16 storage at resolution levels 2-4 (64..1024 ch, 128^2..32^2), fp16 at levels 0-1 "
                 "(512^2, 256^2); fp32 accumulation; " + HEAD16,
        "bf16": "bf16 storage, fp32 accumulation; " + HEAD16, "fp16": "fp16 storage, fp32 accumulation; " + HEAD16,
        "fp32": "fp32 storage and weights, every product as three bf16 terms per operand (6 bf16 MFMA products, fp32 "
                "accumulation: fp32 accuracy), fp32 head",
        "fp32_exact": "fp32 (exact-fp32 MFMA), fp32 head"}
STRONG_GLOBAL = (256, 1024)   # north_star's batch 256 and BASELINE config 4's batch 1024

# launch order of include/unet_mi355x.h: (name, cin, cout, input level, kind); the kernel
# instantiation of each launch comes from the library (unet_launch_label)
LAUNCHES = [
    ("down1.0", None, 64, 0, "first"),
    ("down1.3", 64, 64, 0, "c3"),
    ("down2.0", 64, 128, 1, "c3"),
    ("down2.3", 128, 128, 1, "c3"),
    ("down3.0", 128, 256, 2, "c3"),
    ("down3.3", 256, 256, 2, "c3"),
    ("down4.0", 256, 512, 3, "c3"),
    ("down4.3", 512, 512, 3, "c3"),
    ("bottleneck.0", 512, 1024, 4, "c3"),
    ("bottleneck.3", 1024, 1024, 4, "c3"),
    ("up4", 1024, 512, 4, "up"),
    ("conv4.0", 1024, 512, 3, "c3"),
    ("conv4.3", 512, 512, 3, "c3"),
    ("up3", 512, 256, 3, "up"),
    ("conv3.0", 512, 256, 2, "c3"),
    ("conv3.3", 256, 256, 2, "c3"),
    ("up2", 256, 128, 2, "up"),
    ("conv2.0", 256, 128, 1, "c3"),
    ("conv2.3", 128, 128, 1, "c3"),
    ("up1", 128, 64, 1, "up"),
    ("conv1.0", 128, 64, 0, "c3"),
    ("conv1.3", 64, 64, 0, "c3"),
]
TYPE_CODE = {"float": "f", "__bf16": "DF16b", "_Float16": "DF16_"}


def mangled(label):
    """Itanium-mangled symbol of a "kernel<args>" label (what rocprofv3 may print): template
    arguments are element types or ints, the kernel takes one IgemmArgs."""
    m = re.match(r"(\w+)<(.+)>$", label)
    if not m:
        return None
    args = ""
    for tok in (t.strip() for t in m.group(2).split(",")):
        if tok in TYPE_CODE:
            args += TYPE_CODE[tok]
        elif re.fullmatch(r"-?\d+", tok):
            args += f"Li{tok}E"
        else:
            return None
    name = m.group(1)
    return f"_ZN4unet{len(name)}{name}I{args}EEvNS_9IgemmArgsE"


def launch_flops(entry, n, h, w, c_in, ncls=3):
    """Algorithmic FLOPs (2 per MAC) of one layer over n images of h x w."""
    name, cin, cout, lvl, kind = entry
    hh, ww = h >> lvl, w >> lvl
    if kind == "first":
        return 2.0 * 9 * c_in * cout * hh * ww * n
    if kind == "up":   # input at level lvl, output at lvl-1: every input pixel -> 4 outputs
        return 2.0 * cin * 4 * cout * hh * ww * n
    f = 2.0 * 9 * cin * cout * hh * ww * n
    if name == "conv1.3":
        f += 2.0 * 64 * ncls * hh * ww * n     # fused 1x1 out_conv
    return f


def launch_bytes(entry, n, h, w, c_in, esize, ncls=3):
    """Algorithmic HBM bytes of one layer as its own launch: every activation read once and
    written once, weights read once, concat zero-copy, BN/ReLU/pool/head fused."""
    name, cin, cout, lvl, kind = entry
    hh, ww = h >> lvl, w >> lvl
    if kind == "first":
        return n * c_in * hh * ww * 4 + n * hh * ww * cout * esize + 9 * c_in * 64 * 4
    if kind == "up":
        return n * hh * ww * cin * esize + cin * 4 * cout * esize + n * 4 * hh * ww * cout * esize
    b = n * hh * ww * cin * esize + 9 * cin * cout * esize
    if name == "conv1.3":
        return b + n * ncls * hh * ww // 8            # bit-packed masks only
    b += n * hh * ww * cout * esize
    if name.startswith("down") and name.endswith(".3"):
        b += n * (hh // 2) * (ww // 2) * cout * esize  # fused max-pool output
    return b


def launch_table(labels, n, h, w, c_in, esize, ncls=3):
    """Per launch slot: (layer name, kernel label, FLOPs, algorithmic bytes, issues a dispatch).

    Fusions move work between slots so that no slot is credited with work its kernel does not do:
      * slot 0 = x_to_px4 (16-bit plans): the input pre-cast only (fp32 NCHW read, C -> 4
        channels at esize written); down1.0's FLOPs and weights go to the fused down1.3, which
        reads the 4-channel input instead of a 64-channel map;
      * an empty label (up1 inside conv2.3): the ConvTranspose's FLOPs and its weight + output
        bytes go to the previous launch, whose own output (up1's input) never reaches HBM."""
    rows = []
    for entry, lab in zip(LAUNCHES, labels):
        f = launch_flops(entry, n, h, w, c_in, ncls)
        b = launch_bytes(entry, n, h, w, c_in, esize, ncls)
        rows.append([entry[0], lab, f, b, bool(lab)])
    if labels[0].startswith("x_to_px4"):
        rows[1][2] += rows[0][2]
        rows[1][3] += 9 * c_in * 64 * esize - n * h * w * 64 * esize + n * h * w * 4 * esize
        rows[0][2] = 0.0
        rows[0][3] = n * c_in * h * w * 4 + n * h * w * 4 * esize
    for i, r in enumerate(rows):
        if not r[4] and i > 0:    # fused into the previous launch
            _, cin, _, lvl, _ = LAUNCHES[i]
            prev = rows[i - 1]
            prev[2] += r[2]
            # its input (the previous launch's output) is neither written nor read again
            prev[3] += r[3] - 2 * n * (h >> lvl) * (w >> lvl) * cin * esize
            r[1], r[2], r[3] = prev[1], 0.0, 0
    return [tuple(r) for r in rows]


def gen_pages(seed, batch, size, channels, unique=32):
    """Synthetic invoice pages; `unique` distinct pages tiled to the batch (generation cost)."""
    u = max(1, min(unique, batch))
    pages = syn.invoice_pages(seed, u, size, size, channels)
    reps = (batch + u - 1) // u
    return np.ascontiguousarray(np.concatenate([pages] * reps, axis=0)[:batch])


def host_cores():
    """(threads to use, description) of this host's CPU share: the affinity mask, capped by the
    cgroup CPU quota when one is set (on the GPU box os.cpu_count() shows the whole machine)."""
    total = os.cpu_count() or 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    use = min(avail, quota) if quota else avail
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return use, {"os_cpu_count": total, "affinity": avail, "cgroup_quota": quota, "cpu_model": model}


# ----------------------------------------------------------------------------- launching
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n, argv, timeout=None):
    """Run this script as n rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, the
    torchrun contract) and return the worst exit code.  The caller has made no GPU call (a process
    that initialised the GPU must not hand over to others, and the ranks pick their own device).
    If one rank fails the others are stopped (their exact PIDs), so a lost peer cannot hang the job."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    t0, rcs, first_bad = time.time(), [None] * n, None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0) and first_bad is None:
                    first_bad = rcs[i]     # the root cause, not the peers stopped below
        if first_bad is not None or (timeout and time.time() - t0 > timeout):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                try:
                    rcs[i] = p.wait(timeout=30) if rcs[i] is None else rcs[i]
                except subprocess.TimeoutExpired:
                    p.kill()
                    rcs[i] = p.wait()
            break
        time.sleep(0.05)
    if first_bad is not None:
        return first_bad if first_bad > 0 else 128 - first_bad    # a signal -> 128 + signum
    return 0 if all(rc == 0 for rc in rcs) else 124                # timed out


# ----------------------------------------------------------------------------- per-rank runners
class NativeRunner:
    """The product path: UNet on the native library, forward of a shard into bit-packed masks."""

    def __init__(self, args, dev, world):
        from unet_mi355x import native
        from unet_mi355x.model import UNet
        self.native, self.dev, self.args = native, dev, args
        C = args.channels
        # weights: the real checkpoint is an LFS pointer, so the seeded synthetic weights with the
        # fine-tuned BN/bias subset ("pretrained", tools/pretrain_synthetic.py) that gives a
        # trained-like bimodal logit distribution; "structured" = the untrained seeded weights with
        # the out_conv bias re-centred so that ~10% of each field's pixels pass its threshold.
        self.sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, C, 3, args.weights).items()}
        self.model = self.make_model(args.dtype)
        self.world = world
        self.stream = torch.cuda.current_stream(dev).cuda_stream

    def make_model(self, dtype):
        from unet_mi355x.model import UNet
        m = UNet(self.args.channels, 3, compute_dtype=dtype)
        m.load_state_dict(self.sd)
        return m.to(self.dev).eval()

    def recentre(self, x):
        """'structured' weights: shift the out_conv bias so ~10 % of each field passes (all ranks equal)."""
        with torch.no_grad():   # full-batch forward: every profiled dispatch has the timed shape
            lg = self.model(x)[:2]
        thr = torch.tensor([0.25, 0.40, 0.30], dtype=torch.float64)
        q = torch.quantile(lg.double().transpose(0, 1).reshape(3, -1).cpu(), 0.9, dim=1)
        del lg
        shift = (torch.log(thr / (1 - thr)) - q).float()
        if self.world > 1:
            shift = shift.to(self.dev)
            dist.broadcast(shift, 0)
            shift = shift.cpu()
        with torch.no_grad():
            self.model.out_conv.bias.add_(shift.to(self.dev))
        self.sd = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def handle(self, model=None):
        return (model or self.model).native_handle(self.dev)

    def reserve(self, n, s, model=None):
        self.handle(model).reserve(n, s, s)

    def segment_fn(self, model=None):
        h, stream, bits = self.handle(model), self.stream, self.native.MASK_BITS

        def segment(x_local, masks_local):
            h.forward(x_local, None, masks_local, bits, stream)
        return segment


class StandinRunner:
    """CPU stand-in for the per-rank forward (tests/test_dist_cpu.py drives bench.py with it under
    gloo): a deterministic function of each image into the bit-packed mask shape."""

    def __init__(self, args, dev, world):
        self.dev, self.world = dev, world

    def reserve(self, n, s, model=None):
        pass

    def segment_fn(self, model=None):
        def segment(x_local, masks_local):
            v = x_local.sum(dim=(1, 2, 3)).abs().floor().to(torch.uint8)
            masks_local.copy_((v.view(-1, 1, 1, 1) + torch.arange(masks_local.shape[-1], dtype=torch.uint8)
                               ).expand_as(masks_local))
        return segment


def make_leg(runner, rank, world, n_total, per_rank, seed, S, C, dev, chunk, collective=None):
    """Buffers of one timed configuration on this rank: its input shard, its mask shard inside the
    preallocated all-gather send buffer, and the step function (forward + the one exchange).  A
    shard larger than ``chunk`` images runs as consecutive forwards of at most ``chunk`` (the
    workspace is sized for ``chunk``: 194 MB per 512^2 image at 16 bits).  ``step(ev)`` records the
    event pair ``ev`` (when given) around the exchange: the all-gather's own time inside the step."""
    if per_rank is not None:                        # weak scaling: every rank holds per_rank images
        lo, hi = rank * per_rank, (rank + 1) * per_rank
        n_total = world * per_rank
    else:
        lo, hi = udist.shard_bounds(n_total, rank, world)
    n_local = hi - lo
    x = torch.from_numpy(gen_pages(seed + rank, max(n_local, 1), S, C)).to(dev)[:n_local]
    gather = udist.MaskGather(n_total, (3, S, S // 8), torch.uint8, dev, rank=rank, world=world,
                              collective=collective)
    segment = runner.segment_fn()

    def step(ev=None):
        if n_local <= chunk and ev is None:   # the library's data-parallel step (tests/test_dist_cpu.py drives it too)
            udist.sharded_mask_step(segment, x, gather)
            return
        for i in range(0, n_local, chunk):
            segment(x[i:i + chunk], gather.local[i:i + chunk])
        if ev is not None:
            ev[0].record()
        gather()
        if ev is not None:
            ev[1].record()
    return {"x": x, "gather": gather, "step": step, "n_total": n_total, "n_local": n_local}


class HostMark:
    """torch.cuda.Event's record / elapsed_time on the host clock: the CPU stand-in's per-step marks."""

    def __init__(self):
        self.t = None

    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return 1e3 * (other.t - self.t)


def time_leg(leg, steps, warmup, sync, dev, per_step_events=False):
    """The bench contract's timing loop (udist.timed_steps): barrier + sync on both sides, the MAX
    over ranks; optional per-step GPU times (HIP events on this stream; host marks for the CPU
    stand-in) as a diagnostic, and -- when the leg's step runs the collective -- the all-gather's own
    time per step (marks around it) and this rank's compute time per step (step start to the
    all-gather: its forwards)."""
    # no Python garbage collection inside the timed steps (timeit's practice): a collection pass over
    # torch's and numpy's objects pauses the launching thread for milliseconds, and the GPU idles
    gc.collect()
    gc_was_enabled = gc.isenabled()
    gc.disable()
    ev = ag = None
    collective = "gather" in leg and leg["gather"].collective   # the secondary legs have no exchange
    if per_step_events:
        # created and recorded once before the warmup: torch creates the HIP events lazily at their first
        # record, which would otherwise happen inside the timed steps
        mark = HostMark if dev.type == "cpu" else (lambda: torch.cuda.Event(enable_timing=True))
        ev = [mark() for _ in range(steps + 1)]
        if collective:
            ag = [(mark(), mark()) for _ in range(steps)]
        for e in ev + [e for pair in (ag or ()) for e in pair]:
            e.record()
    for _ in range(warmup):
        leg["step"]()
    marks = iter(ev[1:]) if ev else iter(())
    ag_marks = iter(ag) if ag else iter(())

    first = [bool(ev)]

    def timed_step():
        if first[0]:   # step 0's start mark inside the timed region (after timed_steps' barrier + sync),
            first[0] = False   # so a rank's compute time never includes the wait at that barrier
            ev[0].record()
        pair = next(ag_marks, None)
        if pair is None:
            leg["step"]()
        else:
            leg["step"](pair)
        e = next(marks, None)
        if e is not None:
            e.record()
    try:
        elapsed, host = udist.timed_steps(timed_step, steps, 0, sync=sync, device=dev, collective=collective)
    finally:
        if gc_was_enabled:
            gc.enable()
    out = {"elapsed": elapsed, "ms_per_step": 1e3 * elapsed / steps,
           "value": leg["n_total"] * steps / elapsed, "host_step_ms": [round(1e3 * t, 3) for t in host]}
    if ev:
        out["step_ms"] = [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(steps)]
        # this rank's forwards per step: the whole step without an exchange, else up to the all-gather
        out["compute_ms"] = out["step_ms"] if not ag else \
            [round(ev[i].elapsed_time(ag[i][0]), 3) for i in range(steps)]
    if ag:
        out["allgather_ms"] = [round(a.elapsed_time(b), 4) for a, b in ag]
    return out


def over_ranks(v, dev):
    """(max, min) of a per-rank scalar over the ranks (one all-reduce each; v itself at world 1)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return v, v
    t = torch.tensor([v, -v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0].item()), -float(t[1].item())


# ----------------------------------------------------------------------------- measurement legs
def kernel_table(runner, model, x, masks, B, S, C, dtype, traffic_json):
    """Per-launch HIP-event timing (unet_forward_timed, on the launch stream) -> per-instantiation
    totals and the dominant kernel's roofline."""
    native = runner.native
    h = runner.handle(model)
    labels = h.launch_labels()
    ms = h.forward_timed(x, None, masks, native.MASK_BITS, runner.stream)
    esize = 4 if dtype.startswith("fp32") else 2
    kernels, layer_ms = {}, {}
    for (layer, lab, f, b, own), t in zip(launch_table(labels, B, S, S, C, esize), ms):
        layer_ms[layer] = round(t, 3)
        k = kernels.setdefault(lab, {"launches": 0, "ms": 0.0, "gflop": 0.0, "algo_gb": 0.0, "layers": []})
        k["launches"] += 1 if own else 0
        k["ms"] += t
        k["gflop"] += f / 1e9
        k["algo_gb"] += b / 1e9
        k["layers"].append(layer)
        if not own:   # issues no dispatch of its own (tools/pmc_summary.py)
            k.setdefault("fused_layers", []).append(layer)
    dom_name, dom = max(((n, k) for n, k in kernels.items() if k["gflop"] > 0 and "first_conv" not in n),
                        key=lambda kv: kv[1]["ms"])
    achieved = dom["gflop"] / dom["ms"]   # TFLOP/s (GFLOP / ms)
    for k in kernels.values():
        k["tflops"] = round(k["gflop"] / k["ms"], 1) if k["ms"] > 0 else None
        k["algo_gbs"] = round(k["algo_gb"] / k["ms"] * 1e3, 1) if k["ms"] > 0 else None
        k["avg_launch_ms"] = round(k["ms"] / max(1, k["launches"]), 4)
        k["ms"] = round(k["ms"], 3)
        k["gflop"] = round(k["gflop"], 1)
        k["algo_gb"] = round(k["algo_gb"], 3)
    peak = PEAK_TFLOPS[dtype]
    traffic, source = None, {}
    if traffic_json == "auto":
        traffic_json = os.path.join(REPO, "profiles", f"pmc_{dtype}_bs{B}" + ("" if S == 512 else f"_{S}") + ".json")
    if traffic_json and os.path.exists(traffic_json):
        tj = json.load(open(traffic_json))
        traffic = tj.get(dom_name, {}).get("hbm_bytes_per_launch")
        meta = tj.get("_meta", {})
        from unet_mi355x.native import kernel_sources_sha256
        stamped = meta.get("kernel_sources_sha256")
        # scalars (the driver's record keeps roofline's scalar fields): where the PMC bytes come from and
        # whether they describe the kernels timed here (None: not stamped, an older summary)
        source = {"traffic_file": os.path.relpath(traffic_json, REPO), "traffic_commit": meta.get("source_commit"),
                  "traffic_collected": meta.get("collected"), "traffic_kernel_sources_sha256": stamped,
                  "kernel_sources_match": None if stamped is None else stamped == kernel_sources_sha256()}
    roofline = {"bound": "mfma", "kernel": dom_name, "symbol": mangled(dom_name),
                "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_over_algo": round(traffic / (dom["algo_gb"] * 1e9 / dom["launches"]), 3) if traffic else None,
                **source,
                "launches_per_step": dom["launches"], "avg_launch_ms": dom["avg_launch_ms"],
                "gflop_per_launch": round(dom["gflop"] / dom["launches"], 1),
                "algo_bytes_per_launch": round(dom["algo_gb"] * 1e9 / dom["launches"])}
    roofline.update(min_3x3(labels, ms, B, S, C, peak))
    total_gflop = sum(launch_flops(e, B, S, S, C) for e in LAUNCHES) / 1e9
    return kernels, layer_ms, roofline, total_gflop, sum(ms)


def min_3x3(labels, ms, n, s, c_in, peak):
    """north_star's "≥ 40 % of MFMA peak on the 3x3 DoubleConv layers" as scalars: per launch that runs a
    3x3 layer (HIP-event time of that launch), its 3x3 FLOPs / time / peak, and the minimum over them.
    ``min_3x3_frac`` credits a launch with every 3x3 conv it runs (down1.0 inside the fused down1.3 launch
    of the 16-bit plans) and nothing else (the fused up1 ConvTranspose and the 1x1 head are left out);
    ``min_3x3_frac_own`` credits it with its own layer only (down1.3 without down1.0)."""
    fused_first = labels[0].startswith("x_to_px4")
    best = (None, 9.0, 9.0)
    for i, (entry, lab, t) in enumerate(zip(LAUNCHES, labels, ms)):
        if entry[4] != "c3" or not lab or t <= 0:
            continue
        name, cin, cout, lvl, _ = entry
        own = 2.0 * 9 * cin * cout * (s >> lvl) * (s >> lvl) * n
        f = own + (launch_flops(LAUNCHES[0], n, s, s, c_in) if i == 1 and fused_first else 0.0)
        frac, frac_own = f / (t * 1e9) / peak, own / (t * 1e9) / peak
        if frac < best[1]:
            best = (name, frac, frac_own)
    if best[0] is None:
        return {}
    return {"min_3x3_layer": best[0], "min_3x3_frac": round(best[1], 4), "min_3x3_frac_own": round(best[2], 4)}


def cpu_baseline(args, sd, x, masks, C, S, extra=()):
    """The oracle (fp32 eager torch restating unet_model.py / inference.py) on this host's
    cores: batch-1 forward (images/s + the mask IoU of the GPU masks), batch-8 forward, and
    run_unet end to end (model load + resize + forward + masks + crops, inference.py:50-129).
    extra: (name, x [n, C, h, w] CPU, bit-packed GPU masks [n, 3, h, w/8] CPU, GPU dtype) of other
    legs, whose masks are compared with the oracle's as `<name>_iou_min` / `_mean` / `_images`."""
    from PIL import Image
    from oracle import unet_oracle as orc
    threads, info = host_cores()
    torch.set_num_threads(threads)
    sd_cpu = {k: v.detach().cpu() for k, v in sd.items()}
    xc = x[:64].cpu()
    mk = np.unpackbits(masks[:64].cpu().numpy(), axis=-1, bitorder="little").astype(bool)
    orc.unet_forward(sd_cpu, xc[:1, :, :64, :64])  # warm the CPU kernels
    done, ious, t0 = 0, [], time.perf_counter()
    while done < xc.shape[0] and (done == 0 or time.perf_counter() - t0 < args.cpu_seconds):
        lg = orc.unet_forward(sd_cpu, xc[done:done + 1]).numpy()[0]
        ref = orc.masks_from_logits(lg)
        ious += [orc.mask_iou(mk[done, i], ref[f]) for i, f in enumerate(orc.FIELDS)]
        done += 1
    t_bs1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    orc.unet_forward(sd_cpu, xc[:8])
    t_bs8 = time.perf_counter() - t0
    # run_unet on a 600x400 photo, checkpoint re-loaded on every call as the reference does
    page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
    pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save(sd_cpu, ck)
        lat = []
        for _ in range(2):
            t0 = time.perf_counter()
            orc.run_unet(pil, ck)
            lat.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        orc.load_model_state(ck)
        t_load = time.perf_counter() - t0
    more = {}
    for name, xe, me, dte in extra:
        ie = []
        for j in range(xe.shape[0]):
            ref = orc.masks_from_logits(orc.unet_forward(sd_cpu, xe[j:j + 1]).numpy()[0])
            got = np.unpackbits(me.numpy()[j], axis=-1, bitorder="little").astype(bool)
            ie += [orc.mask_iou(got[i], ref[f]) for i, f in enumerate(orc.FIELDS)]
        more.update({f"{name}_iou_min": round(min(ie), 5), f"{name}_iou_mean": round(float(np.mean(ie)), 5),
                     f"{name}_iou_images": int(xe.shape[0]), f"{name}_iou_size": int(xe.shape[-1]),
                     f"{name}_iou_gpu_dtype": dte})
    # scalars only: the driver's record keeps the scalar fields of cpu_baseline / roofline
    return {"value": round(done / t_bs1, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{done} of the bench images, batch 1, {S}x{S}, fp32 eager torch (oracle/unet_oracle.py), "
                      f"{threads} threads",
            "host_cpu": info["cpu_model"], "host_os_cpu_count": info["os_cpu_count"],
            "host_affinity": info["affinity"], "host_cgroup_quota": info["cgroup_quota"],
            "bs8_images_per_s": round(8 / t_bs8, 4),
            "run_unet_s": round(float(np.median(lat)), 3), "model_load_s": round(t_load, 3),
            "run_unet_sample": "600x400 RGB photo, 2 calls, checkpoint re-loaded per call (inference.py:58)",
            # the headline's quality: GPU masks of the timed batch against the oracle's (inference.py:72-79)
            "iou_min": round(min(ious), 5), "iou_mean": round(float(np.mean(ious)), 5), "iou_images": done,
            "iou_fields": len(ious), "iou_gpu_dtype": args.dtype, **more}


def fp32_leg(args, runner, dev):
    """BASELINE config 2: a batch-32 512^2 fp32 forward on one GPU -- the reference's precision and
    the drop-in's default (unet_mi355x/model.py DEFAULT_DTYPE) -- timed like the headline (HIP
    events per launch for the roofline against the 157.3 TF fp32 MFMA peak)."""
    B, S, C = args.fp32_batch, 512, args.channels
    model = runner.make_model("fp32")
    runner.reserve(B, S, model)
    x = torch.from_numpy(gen_pages(2000, B, S, C)).to(dev)
    masks = torch.empty((B, 3, S, S // 8), dtype=torch.uint8, device=dev)
    seg = runner.segment_fn(model)
    leg = {"step": lambda: seg(x, masks), "n_total": B}
    t = time_leg(leg, args.fp32_steps, 2, torch.cuda.synchronize, dev)
    kernels, layer_ms, roof, gflop, _ = kernel_table(runner, model, x, masks, B, S, C, "fp32", "auto")
    out = {"config": f"BASELINE config 2 shape: batch {B}, {S}x{S}, UNet({C},3), fp32 storage, products as three bf16 "
                     "terms per operand on v_mfma_f32_16x16x32_bf16 (fp32 accuracy; peak = bf16 peak / 6), fused "
                     "bit-packed masks",
           "value": round(t["value"], 2), "unit": "images/s", "ms_per_step": round(t["ms_per_step"], 3),
           "steps": args.fp32_steps, "whole_step_tflops": round(gflop / t["ms_per_step"], 1),
           "roofline": roof, "kernels": kernels, "layer_ms": layer_ms}
    model.close()
    del x, masks
    return out


CFG5_IOU_PAGES = 3   # config-5 pages checked against the CPU oracle (~3 s each on 16 threads)


def cfg5_leg(args, runner, dev):
    """BASELINE config 5 on one GPU: the reference's 5-level UNet(3,3) at 1024x1024, fp16 storage with
    fp32 accumulation, 64 images per GPU (config 5's per-rank share of batch 512 over 8 GPUs), fused
    bit-packed masks, timed like the headline (HIP events per launch for the roofline; traffic from
    profiles/pmc_fp16_bs64_1024.json).  Returns (summary, the first CFG5_IOU_PAGES pages, their masks) for
    the CPU check."""
    B, S, C = args.cfg5_batch, 1024, args.channels
    model = runner.make_model("fp16")
    runner.reserve(B, S, model)
    x = torch.from_numpy(gen_pages(4000, B, S, C, unique=16)).to(dev)
    masks = torch.empty((B, 3, S, S // 8), dtype=torch.uint8, device=dev)
    seg = runner.segment_fn(model)
    leg = {"step": lambda: seg(x, masks), "n_total": B}
    t = time_leg(leg, args.cfg5_steps, 2, torch.cuda.synchronize, dev)
    kernels, layer_ms, roof, gflop, _ = kernel_table(runner, model, x, masks, B, S, C, "fp16", "auto")
    out = {"config": f"BASELINE config 5 shape per GPU: batch {B}, {S}x{S}, UNet({C},3) (5 resolution levels), "
                     "fp16 storage + fp32 accumulation, fused bit-packed masks",
           "value": round(t["value"], 2), "unit": "images/s", "ms_per_step": round(t["ms_per_step"], 3),
           "steps": args.cfg5_steps, "whole_step_tflops": round(gflop / t["ms_per_step"], 1),
           "roofline": roof, "kernels": kernels, "layer_ms": layer_ms}
    page, mk = x[:CFG5_IOU_PAGES].cpu(), masks[:CFG5_IOU_PAGES].cpu()   # distinct pages (unique=16)
    model.close()
    del x, masks
    return out, page, mk


def gpu_latency(args, runner, dev):
    """Batch-1 latency on the GPU at the drop-in default (fp32) and at the bench plan: the drop-in
    run_unet (cached model, GPU preprocessing, fused masks + boxes, host crops; inference.py:50-129)
    and the bare batch-1 forward, eager (22 launches from the host) and as one hipGraph replay."""
    from PIL import Image
    from unet_mi355x import inference as inf
    native = runner.native
    page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
    pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
    inf.DEVICE = str(dev)
    res = {}
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save(runner.sd, ck)
        for dtype in dict.fromkeys(("fp32", args.dtype)):
            out = res[dtype] = {}
            t0 = time.perf_counter()
            inf.run_unet(pil, ck, compute_dtype=dtype)
            out["run_unet_first_call_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
            lat = []
            for _ in range(20):
                t0 = time.perf_counter()
                inf.run_unet(pil, ck, compute_dtype=dtype)
                lat.append(time.perf_counter() - t0)
            out["run_unet_ms"] = round(1e3 * float(np.median(lat)), 3)
            # photos of several sizes: six geometries in rotation, each graph cached after its
            # first call; then more geometries than the photo-graph LRU holds, so every call captures anew
            varied = [pil.resize(sz) for sz in ((600, 400), (640, 480), (800, 600), (500, 700), (1024, 768), (720, 540))]
            for p in varied:
                inf.run_unet(p, ck, compute_dtype=dtype)
            lat = []
            for _ in range(3):
                for p in varied:
                    t0 = time.perf_counter()
                    inf.run_unet(p, ck, compute_dtype=dtype)
                    lat.append(time.perf_counter() - t0)
            out["run_unet_6_geometries_ms"] = round(1e3 * float(np.median(lat)), 3)
            many = [pil.resize((400 + 16 * i, 300 + 12 * i)) for i in range(inf._Staging.MAX_GRAPHS + 4)]
            lat = []
            for _ in range(2):
                for p in many:
                    t0 = time.perf_counter()
                    inf.run_unet(p, ck, compute_dtype=dtype)
                    lat.append(time.perf_counter() - t0)
            out["run_unet_lru_miss_ms"] = round(1e3 * float(np.median(lat)), 3)
            model = inf._cached_model(ck, dtype)
            h = model.native_handle(dev)
            x1 = torch.from_numpy(gen_pages(3, 1, 512, 3)).to(dev)
            m1 = torch.empty((1, 3, 512, 64), dtype=torch.uint8, device=dev)
            h.reserve(1, 512, 512)
            for _ in range(3):
                h.forward(x1, None, m1, native.MASK_BITS, runner.stream)
            torch.cuda.synchronize()
            ref = m1.clone()
            reps = 50
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                h.forward(x1, None, m1, native.MASK_BITS, runner.stream)
            e1.record()
            torch.cuda.synchronize()
            out["forward_bs1_eager_ms"] = round(e0.elapsed_time(e1) / reps, 4)
            # per-layer breakdown of the batch-1 forward (HIP events around every launch slot; a split-K
            # layer's slot holds its partial launch + reduction; up1's slot is empty when fused)
            for _ in range(3):
                lms = h.forward_timed(x1, None, m1, native.MASK_BITS, runner.stream)
            out["forward_bs1_layer_ms"] = {e[0]: round(t, 4) for e, t in zip(LAUNCHES, lms)}
            g = h.graph(x1, None, m1, native.MASK_BITS)
            m1.zero_()
            g.launch(runner.stream)
            torch.cuda.synchronize()
            out["graph_matches_eager"] = bool(torch.equal(m1, ref))
            e0.record()
            for _ in range(reps):
                g.launch(runner.stream)
            e1.record()
            torch.cuda.synchronize()
            out["forward_bs1_graph_ms"] = round(e0.elapsed_time(e1) / reps, 4)
            out["run_unet_over_forward"] = round(out["run_unet_ms"] / out["forward_bs1_eager_ms"], 3)
            g.close()
        inf._cache.clear()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="images per step over all ranks (strong scaling; overrides --batch)")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--dtype", default="mixed", choices=["mixed", "bf16", "fp16", "fp32", "fp32_exact"])
    ap.add_argument("--weights", default="pretrained", choices=["pretrained", "structured"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-layer-profile", action="store_true")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling shapes (global 256 / 1024)")
    ap.add_argument("--strong-global", type=int, nargs="+", default=None,
                    help="global batches of the strong-scaling legs (default 256 1024 at 512x512; tests use small ones)")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 config-2 leg")
    ap.add_argument("--fp32-batch", type=int, default=32)
    ap.add_argument("--fp32-steps", type=int, default=5)
    ap.add_argument("--no-cfg5", action="store_true", help="skip the BASELINE config 5 leg (1024^2 fp16 bs64)")
    ap.add_argument("--cfg5-batch", type=int, default=64)
    ap.add_argument("--cfg5-steps", type=int, default=5)
    ap.add_argument("--standin", action="store_true",
                    help="CPU stand-in forward over gloo (tests: the launcher, sharding and timing without a GPU)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group (nccl; gloo with --standin) and run the N > 1 exchange -- "
                         "RCCL all-gather inside the step, barriers, device MAX all-reduce -- at every world "
                         "size, world size 1 included (the multi-GPU code path on a one-GPU box)")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="where rank 0 writes the full record (per-kernel tables, per-step times); '' = stderr only")
    ap.add_argument("--traffic-json", default="auto",
                    help="PMC summary (tools/pmc_summary.py output) to fill roofline.traffic; 'auto' = "
                         "profiles/pmc_<dtype>_bs<batch>.json when present (collected by tools/gpu_round.sh)")
    args = ap.parse_args()

    # ---- launch: one process per GPU.  Self-spawn before any GPU call when not under torchrun.
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if not args.standin and torch.cuda.device_count() < args.gpus:   # device_count initialises no GPU
            print(f"bench: --gpus {args.gpus} but only {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
            sys.exit(2)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a different GPU count",
              file=sys.stderr)
        sys.exit(2)
    collective = True if args.dist else None      # None: the exchange runs when world > 1
    if (world > 1 or args.dist) and "MASTER_ADDR" not in os.environ:   # --dist at world 1, no launcher
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    if args.standin:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
        if world > 1 or args.dist:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        runner = StandinRunner(args, dev, world)
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        sync = torch.cuda.synchronize
        if world > 1 or args.dist:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)   # RCCL over xGMI
        runner = NativeRunner(args, dev, world)

    if os.environ.get("BENCH_FAIL_RANK") == str(rank):   # tests: a rank dying must fail the whole job
        print(f"bench: rank {rank} failing on request (BENCH_FAIL_RANK)", file=sys.stderr)
        sys.exit(3)
    S, C = args.size, args.channels
    strong = args.global_batch is not None
    legs_cfg = [("main", args.global_batch if strong else None, None if strong else args.batch)]
    strong_global = args.strong_global or (STRONG_GLOBAL if S == 512 else ())
    if not args.no_strong:
        legs_cfg += [(f"strong_{g}", g, None) for g in strong_global if not (strong and g == args.global_batch)]
    chunk = max(args.batch, udist.shard_bounds(args.global_batch, 0, world)[1]) if strong else args.batch
    runner.reserve(chunk, S)

    main_leg = make_leg(runner, rank, world, args.global_batch, None if strong else args.batch, 1000, S, C, dev,
                        chunk, collective)
    B = main_leg["n_local"]
    if not args.standin and args.weights == "structured":
        runner.recentre(main_leg["x"])
        runner.handle()   # re-pack now: the legs' step functions hold this handle and never re-check weights
    res = time_leg(main_leg, args.steps, args.warmup, sync, dev, per_step_events=True)
    # per-rank compute (the forwards of its shard, before the exchange): MAX and MIN over the ranks, so a
    # scaling line splits lost efficiency into compute imbalance and exchange
    comp_max, comp_min = over_ranks(float(np.mean(res["compute_ms"])), dev)

    # ---- strong-scaling shapes (same timing protocol, fewer steps)
    strong_out = []
    for name, g, _ in legs_cfg[1:]:
        leg = make_leg(runner, rank, world, g, None, 3000, S, C, dev, chunk, collective)
        t = time_leg(leg, min(args.steps, 10), 2, sync, dev)
        strong_out.append({"global_batch": g, "per_rank_batch": leg["n_local"] if world == 1 else
                           [udist.shard_bounds(g, r, world)[1] - udist.shard_bounds(g, r, world)[0] for r in range(world)],
                           "value": round(t["value"], 2), "ms_per_step": round(t["ms_per_step"], 3),
                           "steps": min(args.steps, 10)})
        del leg

    # ---- per-launch HIP-event timing (same stream) -> dominant kernel roofline
    kernels, roofline, layer_ms, whole = {}, None, {}, None
    if not args.no_layer_profile and not args.standin and B > 0:
        kernels, layer_ms, roofline, gflop, _ = kernel_table(runner, None, main_leg["x"], main_leg["gather"].local,
                                                             B, S, C, args.dtype, args.traffic_json)
        whole = round(gflop / (res["ms_per_step"]), 1)   # algorithmic TFLOP/s of the timed step
        roofline["whole_step_tflops"] = whole

    # ---- rank 0 at N=1: fp32 config-2 leg, CPU baseline, batch-1 latency
    fp32 = cfg5 = cpu = lat = None
    extra = []
    solo = rank == 0 and world == 1 and not args.standin
    if solo and not args.no_fp32 and S == 512 and not args.dtype.startswith("fp32"):
        fp32 = fp32_leg(args, runner, dev)
    if solo and not args.no_cfg5 and S == 512:
        cfg5, page5, masks5 = cfg5_leg(args, runner, dev)
        extra.append(("cfg5", page5, masks5, "fp16"))
    # the batch-1 latencies before the CPU baseline: that leg's 16 OpenMP threads keep spinning after
    # their parallel regions and slowed the host side of the drop-in call measured right after them
    if solo and not args.no_latency and S == 512 and C == 3:
        lat = gpu_latency(args, runner, dev)
    if solo and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, runner.sd, main_leg["x"], main_leg["gather"].local, C, S, extra)

    if rank == 0:
        exchange = main_leg["gather"].collective
        ag = res.get("allgather_ms")
        out = {
            "metric": METRIC, "value": round(res["value"], 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(res["ms_per_step"], 3),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "bf16+fp16" if args.dtype == "mixed" else args.dtype,
            "data": f"synthetic (seeded invoice-like pages, gray x3; '{args.weights}' seeded weights -- "
                    "the trained checkpoint is an LFS pointer)" if not args.standin else "standin (CPU, gloo)",
            "config": {"workload": f"UNet(n_channels={C}, n_classes=3) forward {S}x{S} + fused sigmoid/"
                                   f"threshold bit-packed masks" + (" + RCCL all-gather" if exchange else ""),
                       "global_batch": main_leg["n_total"], "per_gpu_batch": B, "image": S,
                       "parallelism": f"dp{world}", "exchange": "all_gather_into_tensor" if exchange else None,
                       "precision_plan": PLAN[args.dtype]},
            "allgather_ms": round(float(np.mean(ag)), 4) if ag else None,
            "compute_ms": round(comp_max, 3), "compute_ms_min": round(comp_min, 3),
            "roofline": roofline, "cpu_baseline": cpu,
        }
        if out["roofline"] is not None and ag:
            out["roofline"]["allgather_ms"] = out["allgather_ms"]    # the exchange's share of ms_per_step
        if cpu is not None:    # the secondary legs' headline scalars, where the driver's record keeps them
            for name, leg in (("fp32", fp32), ("cfg5", cfg5)):
                if leg:
                    cpu[f"{name}_images_per_s"] = leg["value"]
                    cpu[f"{name}_ms_per_step"] = leg["ms_per_step"]
                    cpu[f"{name}_frac"] = leg["roofline"]["frac"]
            for dt, l in (lat or {}).items():
                cpu[f"gpu_run_unet_ms_{dt}"] = l["run_unet_ms"]
                cpu[f"gpu_forward_bs1_ms_{dt}"] = l["forward_bs1_eager_ms"]
        # compact summaries of the other legs; the full tables go to the detail record
        out["strong_scaling"] = strong_out
        for name, leg in (("fp32", fp32), ("cfg5", cfg5)):
            out[name] = None if leg is None else {
                k: leg[k] for k in ("config", "value", "unit", "ms_per_step", "steps", "whole_step_tflops")}
            if leg:
                out[name]["roofline"] = {k: leg["roofline"].get(k) for k in
                                         ("kernel", "achieved", "frac", "traffic", "kernel_sources_match")}
        out["latency_bs1"] = None if lat is None else {
            dt: {k: v for k, v in l.items() if k != "forward_bs1_layer_ms"} for dt, l in lat.items()}
        detail = {"step_ms": res.get("step_ms"), "host_step_ms": res["host_step_ms"], "allgather_ms": ag,
                  "compute_ms": res["compute_ms"],
                  "kernels": kernels, "layer_ms": layer_ms, "fp32": fp32, "cfg5": cfg5, "latency_bs1": lat}
        line = json.dumps(out)
        print("bench_detail " + json.dumps(detail), file=sys.stderr, flush=True)
        if args.detail_out:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(args.detail_out)), exist_ok=True)
                with open(args.detail_out, "w") as f:
                    json.dump({"summary": out, "detail": detail}, f)
            except OSError as e:
                print(f"bench: could not write {args.detail_out}: {e}", file=sys.stderr)
        print(line, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
