"""A/B per-layer kernel configurations in ONE process (HIP-event timing per launch).

    python tools/tune.py --dtype bf16 --batch 256 --cands "0:2,15:2,16:1" "0:9,16:9" ...

Each candidate is "<UNET_MI355X_CFG>|<UNET_MI355X_UPCFG>": layer index into the 17 3x3 layers
(or 0..3 = up4..up1 after the '|') : Cfg enum value, see csrc/unet_internal.h.  Prints per-launch ms (median of
--reps timed forwards) for every candidate, interleaved round-robin.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import LAUNCHES, gen_pages, launch_flops  # noqa: E402
from unet_mi355x import native  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cands", nargs="+", default=[""])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3).items()}
    x = torch.from_numpy(gen_pages(5, a.batch, a.size, 3)).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    handles = []
    base_env = dict(os.environ)
    for c in a.cands:
        lc, _, rest = c.partition("|")      # "<3x3 layer overrides>|<up overrides>|K=V;K=V (env)"
        uc, _, env = rest.partition("|")
        os.environ.clear()                  # every candidate starts from the launch environment
        os.environ.update(base_env)
        os.environ["UNET_MI355X_CFG"] = lc
        os.environ["UNET_MI355X_UPCFG"] = uc
        for kv in filter(None, env.split(";")):
            k, _, v = kv.partition("=")
            os.environ[k] = v
        m = UNet(3, 3, compute_dtype=a.dtype)
        m.load_state_dict(sd)
        m = m.to(dev).eval()
        h = m.native_handle(dev)
        h.reserve(a.batch, a.size, a.size)
        handles.append((c, m, h))
    masks = torch.empty((a.batch, 3, a.size, a.size // 8), dtype=torch.uint8, device=dev)
    res = {c: [] for c in a.cands}
    for c, m, h in handles:   # warm-up
        h.forward_timed(x, None, masks, native.MASK_BITS, stream)
    for _ in range(a.reps):
        for c, m, h in handles:
            res[c].append(h.forward_timed(x, None, masks, native.MASK_BITS, stream))
    med = {c: np.median(np.array(v), axis=0) for c, v in res.items()}
    for k, c in enumerate(a.cands):   # the columns' legend (candidates often share a long prefix)
        print(f"c{k}: {c!r}")
    print(f"{'launch':14s}" + "".join(f"{'c' + str(k):>24s}" for k in range(len(a.cands))))
    for i, e in enumerate(LAUNCHES):
        f = launch_flops(e, a.batch, a.size, a.size, 3) / 1e9
        print(f"{e[0]:14s}" + "".join(f"{med[c][i]:10.3f}ms {f / med[c][i]:8.0f}TF " for c in a.cands))
    print(f"{'TOTAL':14s}" + "".join(f"{med[c].sum():10.3f}ms {'':10s} " for c in a.cands))


if __name__ == "__main__":
    main()
