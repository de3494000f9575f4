"""Bitwise A/B of two BUILDS of the library (one per process: the library path is fixed at import).

    UNET_MI355X_LIB=.../libunet_mi355x_base.so python tools/lib_ab.py --save gpurun_out/a.npz
    python tools/lib_ab.py --save gpurun_out/b.npz --compare gpurun_out/a.npz

Runs seeded inputs at a few shapes through every 16-bit plan and saves the logits; with --compare
it reports whether they equal the other build's bit for bit (kernel changes that keep the K order
of every accumulator must).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from unet_mi355x import synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save", required=True)
    ap.add_argument("--compare", default=None)
    ap.add_argument("--dtypes", nargs="+", default=["mixed", "fp16", "bf16"])
    ap.add_argument("--shapes", nargs="+", default=["2x512x512", "3x48x80", "1x256x128"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3).items()}
    out = {}
    for dt in a.dtypes:
        m = UNet(3, 3, compute_dtype=dt)
        m.load_state_dict(sd)
        m = m.to(dev).eval()
        for shp in a.shapes:
            n, h, w = (int(v) for v in shp.split("x"))
            g = torch.Generator().manual_seed(n * 1000 + h + w)
            x = torch.rand(n, 3, h, w, generator=g).to(dev)
            with torch.no_grad():
                out[f"{dt}_{shp}"] = m(x).float().cpu().numpy()
        m.close()
    np.savez(a.save, **out)
    if a.compare:
        ref = np.load(a.compare)
        ok = True
        for k, v in out.items():
            same = np.array_equal(v, ref[k])
            ok &= same
            print(f"{k:22s} bitwise={same} max|d|={np.abs(v - ref[k]).max():.3g}", flush=True)
        print("ALL BITWISE" if ok else "MISMATCH")
        sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
