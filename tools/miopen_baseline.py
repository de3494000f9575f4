"""Optional secondary baseline: the same UNet forward in PyTorch-ROCm eager mode
(MIOpen convolutions, torch ops for BN / ReLU / pool / ConvTranspose / cat) on one MI355X.

Not part of the product path; it only puts the native kernels' throughput next to the vendor
library's on the same GPU, same synthetic weights ("pretrained" profile) and pages.

    python tools/miopen_baseline.py [--batch 64] [--dtype bf16] [--steps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pretrain_synthetic import forward  # noqa: E402  (torch.nn.functional restatement of UNet.forward)
from unet_mi355x import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = False
    sd = syn.make_state_dict(0, 3, 3, "pretrained")
    p = {k: torch.from_numpy(np.asarray(v)).to(dev, dt) for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    for k, v in p.items():
        if v.dim() == 4:
            p[k] = v.contiguous(memory_format=torch.channels_last)
    x = torch.from_numpy(syn.invoice_pages(1000, a.batch, a.size, a.size, 3)).to(dev, dt)
    x = x.contiguous(memory_format=torch.channels_last)
    import threading
    done = threading.Event()

    def heartbeat():   # MIOpen compiles kernels on the first call; keep the run visibly alive
        while not done.wait(30):
            print(f"[miopen_baseline] still running ({time.perf_counter() - t0:.0f} s)", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    threading.Thread(target=heartbeat, daemon=True).start()
    with torch.no_grad():
        forward(p, x)        # first call: MIOpen kernel selection / compilation
        torch.cuda.synchronize()
        t_first = time.perf_counter() - t0
        t0 = time.perf_counter()
        for _ in range(a.steps):
            forward(p, x)
        torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / a.steps
    done.set()
    print(json.dumps({"baseline": "pytorch-rocm eager (MIOpen)", "dtype": a.dtype, "batch": a.batch, "image": a.size,
                      "images_per_s": round(a.batch / dt_s, 2), "ms_per_step": round(1e3 * dt_s, 2),
                      "first_call_s": round(t_first, 1), "torch": torch.__version__}), flush=True)


if __name__ == "__main__":
    main()
