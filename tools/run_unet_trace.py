"""Kernel-level view of run_unet at batch 1 (diagnostic): 50 calls of the drop-in on the bench's 600x400
photo, for rocprofv3 --kernel-trace --stats: which kernels besides the forward the photo graph runs."""
import os
import sys
import tempfile
import time

import numpy as np
import torch
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
from unet_mi355x import inference as inf  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "mixed"
page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
inf.DEVICE = "cuda:0"
with tempfile.TemporaryDirectory() as td:
    ck = os.path.join(td, "best_unet_model.pth")
    torch.save({k: torch.as_tensor(v) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}, ck)
    for _ in range(5):
        inf.run_unet(pil, ck, compute_dtype=dtype)
    torch.cuda.synchronize()
    t = []
    for _ in range(50):
        t0 = time.perf_counter()
        inf.run_unet(pil, ck, compute_dtype=dtype)
        t.append(time.perf_counter() - t0)
    print(f"{dtype}: run_unet median {1e3 * float(np.median(t)):.3f} ms")
