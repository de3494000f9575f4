"""Kernel timeline of the drop-in run_unet at batch 1 (run under rocprofv3 --kernel-trace).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python3 tools/trace_run_unet.py
    python tools/trace_run_unet.py --summarise gpurun_out/trace/run_kernel_trace.csv

Runs 30 run_unet calls (the bench's 600x400 page, pretrained-like weights, mixed plan); --summarise
prints, for the last calls, every dispatch's duration and the idle gap before it, and the per-call
totals (busy, gaps, first-to-last)."""
import argparse
import csv
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))


def run(dtype):
    import torch
    from PIL import Image
    from unet_mi355x import inference as inf, synthetic as syn
    inf.DEVICE = "cuda:0"
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}
    page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
    pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save(sd, ck)
        for _ in range(30):
            inf.run_unet(pil, ck, compute_dtype=dtype)
        torch.cuda.synchronize()


def summarise(path, calls=3):
    from pmc_summary import label_of
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # a call starts with the horizontal resize pass
    starts = [i for i, r in enumerate(rows) if "resample_h" in r["Kernel_Name"]]
    for ci in starts[-calls:]:
        end = next((j for j in starts if j > ci), len(rows))
        seq = rows[ci:end]
        t0 = int(seq[0]["Start_Timestamp"])
        busy = gaps = 0
        prev = None
        print(f"--- call at dispatch {ci}")
        for r in seq:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            busy += (e - s) / 1e3
            gaps += max(gap, 0.0)
            print(f"  {(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  gap {gap:6.1f}  {label_of(r['Kernel_Name'])[:90]}")
            prev = e
        print(f"  busy {busy:.1f} us, gaps {gaps:.1f} us, first-to-last {(prev - t0) / 1e3:.1f} us, {len(seq)} kernels")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarise", default=None)
    ap.add_argument("--dtype", default="mixed")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a.dtype)
