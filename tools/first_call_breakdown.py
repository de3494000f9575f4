"""Cold start of the drop-in (GPU box): torch.load, the module build + assign, the native pack, the
first and second run_unet, per precision plan, in one process (the first plan also pays the library's
code-object load).  Usage: python tools/first_call_breakdown.py"""
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tw-invoice-unet-ocr-llm_amd"))
from PIL import Image  # noqa: E402
from unet_mi355x import inference as inf, native, synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402


def main():
    inf.DEVICE = "cuda:0"
    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    t = time.perf_counter()
    native.load_library()
    print(f"library load {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}
    page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
    pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save(sd, ck)
        for dt in ("mixed", "fp32", "mixed"):
            inf._cache.clear()
            inf._staging.clear()
            t0 = time.perf_counter()
            state = torch.load(ck, map_location="cpu", weights_only=True)
            t1 = time.perf_counter()
            with torch.device(inf.DEVICE):
                m = UNet(3, 3, compute_dtype=dt)
            t2 = time.perf_counter()
            m.load_state_dict({k: v.to(inf.DEVICE) for k, v in state.items()}, assign=True)
            m.eval()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            m._prepack(torch.device(inf.DEVICE), state)
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            inf._cache.clear()
            t5 = time.perf_counter()
            inf.run_unet(pil, ck, compute_dtype=dt)   # load_model + first call
            t6 = time.perf_counter()
            inf.run_unet(pil, ck, compute_dtype=dt)
            t7 = time.perf_counter()
            print(f"{dt}: torch.load {1e3 * (t1 - t0):.1f} ms, build on GPU {1e3 * (t2 - t1):.1f} ms, assign to GPU "
                  f"{1e3 * (t3 - t2):.1f} ms, pack + upload {1e3 * (t4 - t3):.1f} ms | first run_unet (load_model "
                  f"inside) {1e3 * (t6 - t5):.1f} ms, second {1e3 * (t7 - t6):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
