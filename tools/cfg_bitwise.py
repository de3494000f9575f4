"""Bitwise comparison of two per-layer kernel configurations of ONE library build (same process).

    python tools/cfg_bitwise.py "<UNET_MI355X_CFG a>" "<UNET_MI355X_CFG b>" [--dtypes mixed fp16 bf16]

Seeded pages at a few shapes through each configuration; the logits and masks must be equal bit for bit
(configurations of one kernel family accumulate in the same order)."""
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
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--dtypes", nargs="+", default=["mixed", "fp16", "bf16"])
    ap.add_argument("--shapes", nargs="+", default=["2x512x512", "3x48x80", "1x256x128", "5x64x96"])
    a = ap.parse_args()
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}
    ok = True
    for dt in a.dtypes:
        for sh in a.shapes:
            n, h, w = (int(v) for v in sh.split("x"))
            x = torch.from_numpy(syn.invoice_pages(11, n, h, w, 3)).to("cuda:0")
            outs = []
            for cfg in (a.a, a.b):
                os.environ["UNET_MI355X_CFG"] = cfg
                os.environ["UNET_MI355X_KSPLIT"] = "0"
                m = UNet(3, 3, compute_dtype=dt)
                m.load_state_dict(sd)
                m = m.to("cuda:0").eval()
                labels = m.native_handle(torch.device("cuda:0")).launch_labels()
                with torch.no_grad():
                    outs.append((m(x).cpu().numpy(), labels[20]))
                m.close()
            same = np.array_equal(outs[0][0], outs[1][0])
            ok &= same
            print(f"{dt:6s} {sh:10s} bitwise={same} max|d|={np.abs(outs[0][0] - outs[1][0]).max():.3g}  "
                  f"conv1.0: {outs[0][1]} | {outs[1][1]}", flush=True)
    print("ALL BITWISE" if ok else "DIFFERENT")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
