"""Where does the occasional slow first timed step of bench.py come from?

Sets up exactly like bench.py's main leg (NativeRunner, reserve, make_leg), then runs several
trials of [warmup W, synchronize, K steps] with a HIP event after EVERY step (warmup included)
and the host clock beside it, so a stall can be placed: in the warmup or the first timed step,
after the synchronize, at a fixed wall time after the workspace allocation, or anywhere.  The last
trial runs every step through unet_forward_timed (per-launch events) to name the launch that
absorbs a stall.  One JSON line per trial on stdout.

    python tools/first_step_probe.py [--trials 4] [--warmup 3] [--steps 10] [--idle-ms 0]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between the sync and the timed steps")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    args = argparse.Namespace(channels=3, weights="pretrained", dtype="mixed", batch=a.batch)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t_start = time.perf_counter()
    runner = bench.NativeRunner(args, dev, 1)
    runner.reserve(a.batch, 512)
    t_reserve = time.perf_counter()
    leg = bench.make_leg(runner, 0, 1, None, a.batch, 1000, 512, 3, dev, a.batch)
    print(json.dumps({"setup_s": round(t_reserve - t_start, 3),
                      "make_leg_s": round(time.perf_counter() - t_reserve, 3)}), flush=True)
    h = runner.handle()
    x, masks = leg["x"], leg["gather"].local
    for trial in range(a.trials):
        timed = trial == a.trials - 1
        n = a.warmup + a.steps
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 2)]
        for e in ev:
            e.record()
        torch.cuda.synchronize()
        host, per_launch = [], []
        ev[0].record()
        t0 = time.perf_counter()
        for i in range(n):
            if i == a.warmup:
                torch.cuda.synchronize()
                if a.idle_ms:
                    time.sleep(a.idle_ms / 1e3)
                ev[i + 1].record()    # an extra mark: the sync gap is its own interval
            t = time.perf_counter()
            if timed:
                per_launch.append([round(v, 3) for v in h.forward_timed(x, None, masks, runner.native.MASK_BITS,
                                                                         runner.stream)])
            else:
                leg["step"]()
            host.append(round(1e3 * (time.perf_counter() - t), 3))
            ev[i + 2 if i >= a.warmup else i + 1].record()
        torch.cuda.synchronize()
        ms = [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(n + 1)]
        gpu_steps = ms[:a.warmup] + ms[a.warmup + 1:]
        out = {"trial": trial, "since_reserve_s": round(t0 - t_reserve, 3), "warmup_ms": gpu_steps[:a.warmup],
               "sync_gap_ms": ms[a.warmup], "timed_ms": gpu_steps[a.warmup:], "host_ms": host}
        if timed:
            labels = [r[0] for r in bench.LAUNCHES]
            med = [sorted(col)[len(col) // 2] for col in zip(*per_launch)]
            out["per_launch_excess_ms"] = [
                {labels[j]: round(v - med[j], 3) for j, v in enumerate(row) if j < len(labels) and v - med[j] > 0.5}
                for row in per_launch]
            out["per_launch_median_ms"] = dict(zip(labels, med))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
