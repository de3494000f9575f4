"""Bitwise A/B check of kernel configurations (ablation-build variants included) in ONE process.

    UNET_MI355X_LIB=.../libunet_mi355x_abl.so python tools/ab_check.py --dtype mixed --cands "" "1:115,2:115"

Builds one handle per candidate (UNET_MI355X_CFG overrides, see tools/tune.py), runs the same
seeded input through each at a few shapes and reports whether the logits equal the first
candidate's bit for bit (the ring variants keep the K order, so they must).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from unet_mi355x import synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="mixed")
    ap.add_argument("--cands", nargs="+", default=[""])
    ap.add_argument("--shapes", nargs="+", default=["2x512x512", "3x48x80", "1x256x128"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3).items()}
    models = []
    for c in a.cands:
        os.environ["UNET_MI355X_CFG"] = c
        m = UNet(3, 3, compute_dtype=a.dtype)
        m.load_state_dict(sd)
        models.append((c, m.to(dev).eval()))
    ok = True
    for shp in a.shapes:
        n, h, w = (int(v) for v in shp.split("x"))
        g = torch.Generator().manual_seed(n * 1000 + h + w)
        x = torch.rand(n, 3, h, w, generator=g).to(dev)
        with torch.no_grad():
            outs = [m(x).float().cpu() for _, m in models]
        for (c, _), o in zip(models[1:], outs[1:]):
            same = torch.equal(o, outs[0])
            ok &= same
            print(f"{shp:12s} {c[:40]:40s} bitwise={same} max|d|={(o - outs[0]).abs().max().item():.3g}", flush=True)
    print("ALL BITWISE" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
