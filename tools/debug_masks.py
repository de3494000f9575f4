"""Diagnose fused-mask disagreements: u8 masks, bit-packed masks and logits of one forward."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from unet_mi355x import native  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402

dev = torch.device("cuda", 0)
lib = native.load_library()
x = torch.from_numpy(syn.invoice_pages(21, 2, 512, 512, 3)).to(dev)
for dtype in ("fp32", "bf16"):
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(21, 3, 3, profile="structured").items()}
    m = UNet(3, 3, compute_dtype=dtype)
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    with torch.no_grad():
        lg = m(x).cpu().numpy()
        q = np.quantile(lg.transpose(1, 0, 2, 3).reshape(3, -1), 0.9, axis=1)
        thr = np.array([0.25, 0.40, 0.30])
        sd["out_conv.bias"] = sd["out_conv.bias"] + torch.from_numpy((np.log(thr / (1 - thr)) - q).astype(np.float32))
        m.load_state_dict(sd)
        masks, logits = m.forward_masks(x, with_logits=True)
        bits = m.forward_masks(x, packed=True)
    masks = masks.cpu().numpy().astype(bool)
    logits = logits.cpu().numpy()
    unpacked = np.unpackbits(bits.cpu().numpy(), axis=-1, bitorder="little").astype(bool)
    cut = np.array([lib.unet_logit_cut(t) for t in thr], np.float32)
    pred = logits > cut[None, :, None, None]
    for name, a in (("u8", masks), ("bits", unpacked)):
        d = np.argwhere(a != pred)
        print(dtype, name, "mismatches vs logits>cut:", len(d), "of", a.size, "on-frac", a.mean())
        if len(d):
            print("  first", d[:8].tolist())
            print("  y%2", np.bincount(d[:, 2] % 2), "x%16", np.bincount(d[:, 3] % 16, minlength=16))
            print("  classes", np.bincount(d[:, 1], minlength=3))
    m.close()
