"""Run the same forward several times and report the first intermediate that differs bitwise."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from unet_mi355x import native  # noqa: E402
if "prev" in os.environ.get("UNET_MI355X_LIB", ""):
    native.SIGNATURES.pop("unet_logit_cut", None)
from unet_mi355x import synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402

NAMES = ["c1", "p1", "c2", "p2", "c3", "p3", "c4", "p4", "bn", "u4", "c7", "u1", "c8a"]
dev = torch.device("cuda", 0)
n = int(os.environ.get("DBG_N", "2"))
x = torch.from_numpy(syn.invoice_pages(21, n, 512, 512, 3)).to(dev)
for dtype in ("fp32", "bf16"):
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(21, 3, 3, profile="structured").items()}
    m = UNet(3, 3, compute_dtype=dtype)
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    runs = []
    for r in range(4):
        with torch.no_grad():
            lg = m(x)
        torch.cuda.synchronize()
        inter = {k: m.intermediate(k).cpu().numpy() for k in NAMES}
        inter["logits"] = lg.cpu().numpy()
        runs.append(inter)
    for r in range(1, 4):
        bad = [(k, int((runs[r][k] != runs[0][k]).sum()), float(np.abs(runs[r][k] - runs[0][k]).max()))
               for k in NAMES + ["logits"] if not np.array_equal(runs[r][k], runs[0][k])]
        print(dtype, "run", r, "differs:", bad[:6] if bad else "none", flush=True)
    m.close()
