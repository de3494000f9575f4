"""Compare kernel configurations against the defaults, intermediate by intermediate, and
every configuration's logits against the CPU oracle.

    python tools/debug_cfg.py [--dtype bf16] [--size 128] "<UNET_MI355X_CFG>|<UNET_MI355X_UPCFG>" ...
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import unet_oracle as orc  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402

NAMES = ["c1", "p1", "c2", "p2", "c3", "p3", "c4", "p4", "bn", "u4", "u3", "u2", "c7", "u1", "c8a"]


def run(sd, x, dtype, cand):
    lc, _, uc = cand.partition("|")
    os.environ["UNET_MI355X_CFG"] = lc
    os.environ["UNET_MI355X_UPCFG"] = uc
    m = UNet(3, 3, compute_dtype=dtype)
    m.load_state_dict(sd)
    m = m.to(x.device).eval()
    with torch.no_grad():
        lg = m(x)
    torch.cuda.synchronize()
    out = {}
    for k in NAMES:
        try:
            out[k] = m.intermediate(k).float().cpu().numpy()
        except RuntimeError:   # c7 with up1 fused into conv2.3: never stored
            pass
    out["logits"] = lg.cpu().numpy()
    m.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("cands", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sd_np = syn.make_state_dict(3, 3, 3, profile="structured")
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in sd_np.items()}
    xc = torch.from_numpy(syn.invoice_pages(3, a.n, a.size, a.size, 3))
    ref = orc.unet_forward(sd_np, xc).numpy()
    scale = max(1.0, float(np.abs(ref).max()))
    x = xc.to(dev)
    base = run(sd, x, a.dtype, "")
    print(f"default: logits rel err vs oracle {np.abs(base['logits'] - ref).max() / scale:.3e}")
    for c in a.cands:
        o = run(sd, x, a.dtype, c)
        err = np.abs(o["logits"] - ref).max() / scale
        print(f"cand {c!r}: logits rel err vs oracle {err:.3e}")
        for k in [n for n in NAMES if n in o and n in base] + ["logits"]:
            d = np.abs(o[k] - base[k])
            if d.max() > 0:
                idx = np.unravel_index(np.argmax(d), d.shape)
                print(f"   {k:7s} shape {o[k].shape} differing {int((d > 0).sum())} max {d.max():.4g} at {idx}")


if __name__ == "__main__":
    main()
