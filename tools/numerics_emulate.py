"""CPU emulation of the native path's storage precision, per layer (tool, not a test).

Restates the native forward's rounding points on the CPU: BN folded in fp64 then rounded to
the layer's storage type, the network input rounded to the first layer's type (x_to_px4),
every conv / ConvTranspose output rounded to the storage type of its consumer, fp32
accumulation, the fused head on the fp32 conv1.3 accumulators.  Compares the fused masks
with the fp32 oracle masks (inference.py:72-79) on the bench's page sample, so a per-layer
precision plan can be chosen before any kernel is written.

    python tools/numerics_emulate.py --images 26 --plans bf16 fp16 bf16_l0dec16
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import unet_oracle as orc  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402

LAYERS = ["down1.0", "down1.3", "down2.0", "down2.3", "down3.0", "down3.3", "down4.0", "down4.3",
          "bottleneck.0", "bottleneck.3", "up4", "conv4.0", "conv4.3", "up3", "conv3.0", "conv3.3",
          "up2", "conv2.0", "conv2.3", "up1", "conv1.0", "conv1.3"]
TD = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def plan_of(name: str) -> dict:
    """layer -> storage dtype of its weights and of its INPUT operand (what its MFMA reads).
    "base+layer=dt,layer=dt": a named plan with per-layer overrides (e.g. "lv01+down1.0=bf16")."""
    if "+" in name:
        base, _, ov = name.partition("+")
        p = plan_of(base)
        for item in ov.split(","):
            k, _, dt = item.partition("=")
            if k not in p or dt not in TD:
                raise ValueError(item)
            p[k] = dt
        return p
    p = {k: "bf16" for k in LAYERS}
    if name == "fp16":
        p = {k: "fp16" for k in LAYERS}
    elif name == "bf16_l0dec16":        # cat1 (up1 + c1 skip), conv1.0, conv1.3 in fp16
        for k in ("conv1.0", "conv1.3"):
            p[k] = "fp16"
    elif name == "bf16_l0dec16_up1":    # + up1 computed in fp16 (reads c7 in fp16)
        for k in ("conv1.0", "conv1.3", "up1"):
            p[k] = "fp16"
    elif name == "bf16_c13":
        p["conv1.3"] = "fp16"
    elif name == "bf16_in16":           # input + first conv in fp16
        p["down1.0"] = "fp16"
        p["down1.3"] = "fp16"
    elif name == "bf16_l0":             # whole level 0 (encoder and decoder) fp16
        for k in ("down1.0", "down1.3", "conv1.0", "conv1.3"):
            p[k] = "fp16"
    elif name == "bf16_l01dec":
        for k in ("conv1.0", "conv1.3", "up1", "conv2.0", "conv2.3"):
            p[k] = "fp16"
    elif name.startswith("lv"):         # "lv01": every layer whose INPUT is at the listed levels in fp16
        lv = {"down1.0": 0, "down1.3": 0, "down2.0": 1, "down2.3": 1, "down3.0": 2, "down3.3": 2, "down4.0": 3,
              "down4.3": 3, "bottleneck.0": 4, "bottleneck.3": 4, "up4": 4, "conv4.0": 3, "conv4.3": 3, "up3": 3,
              "conv3.0": 2, "conv3.3": 2, "up2": 2, "conv2.0": 1, "conv2.3": 1, "up1": 1, "conv1.0": 0, "conv1.3": 0}
        keep = {int(ch) for ch in name[2:]}
        for k in LAYERS:
            if lv[k] in keep:
                p[k] = "fp16"
    elif name != "bf16":
        raise ValueError(name)
    return p


def rnd(x, dt):
    return x.to(TD[dt]).to(torch.float32)


def fold(sd, blk, ci):
    bn = str(int(ci) + 1)
    w = torch.from_numpy(np.asarray(sd[f"{blk}.net.{ci}.weight"])).double()
    b = torch.from_numpy(np.asarray(sd[f"{blk}.net.{ci}.bias"])).double()
    g = torch.from_numpy(np.asarray(sd[f"{blk}.net.{bn}.weight"])).double()
    be = torch.from_numpy(np.asarray(sd[f"{blk}.net.{bn}.bias"])).double()
    mu = torch.from_numpy(np.asarray(sd[f"{blk}.net.{bn}.running_mean"])).double()
    var = torch.from_numpy(np.asarray(sd[f"{blk}.net.{bn}.running_var"])).double()
    s = g / torch.sqrt(var + 1e-5)
    return (w * s[:, None, None, None]).float(), ((b - mu) * s + be).float()


def emulate(sd, x, plan, head=None):
    """Logits of the emulated native forward (fp32 NCHW).  head = "fp16" / "bf16": the 1x1 head's
    operands (conv1.3's ReLU outputs and the out_conv weights) rounded to that type, fp32
    accumulation and bias (a head on 16-bit MFMAs); None: the fp32 head."""
    def conv(name, h, out_dt):
        blk, ci = name.split(".")
        w, b = fold(sd, blk, ci)
        dt = plan[name]
        y = F.relu(F.conv2d(rnd(h, dt), rnd(w, dt), b, padding=1))
        return y if out_dt is None else rnd(y, out_dt)

    def upc(name, h, out_dt):
        w = torch.from_numpy(np.asarray(sd[f"{name}.weight"]))
        b = torch.from_numpy(np.asarray(sd[f"{name}.bias"]))
        dt = plan[name]
        return rnd(F.conv_transpose2d(rnd(h, dt), rnd(w, dt), b, stride=2), out_dt)

    P = plan
    with torch.no_grad():
        a = conv("down1.0", x, P["down1.3"])
        c1 = conv("down1.3", a, None)
        c1s = rnd(c1, P["conv1.0"])                 # skip into cat1 (conv1.0's operand type)
        p1 = rnd(F.max_pool2d(c1, 2), P["down2.0"])
        a = conv("down2.0", p1, P["down2.3"])
        c2 = conv("down2.3", a, None)
        c2s, p2 = rnd(c2, P["conv2.0"]), rnd(F.max_pool2d(c2, 2), P["down3.0"])
        a = conv("down3.0", p2, P["down3.3"])
        c3 = conv("down3.3", a, None)
        c3s, p3 = rnd(c3, P["conv3.0"]), rnd(F.max_pool2d(c3, 2), P["down4.0"])
        a = conv("down4.0", p3, P["down4.3"])
        c4 = conv("down4.3", a, None)
        c4s, p4 = rnd(c4, P["conv4.0"]), rnd(F.max_pool2d(c4, 2), P["bottleneck.0"])
        a = conv("bottleneck.0", p4, P["bottleneck.3"])
        bn = conv("bottleneck.3", a, P["up4"])
        u = torch.cat([upc("up4", bn, P["conv4.0"]), c4s], 1)
        a = conv("conv4.0", u, P["conv4.3"])
        c5 = conv("conv4.3", a, P["up3"])
        u = torch.cat([upc("up3", c5, P["conv3.0"]), c3s], 1)
        a = conv("conv3.0", u, P["conv3.3"])
        c6 = conv("conv3.3", a, P["up2"])
        u = torch.cat([upc("up2", c6, P["conv2.0"]), c2s], 1)
        a = conv("conv2.0", u, P["conv2.3"])
        c7 = conv("conv2.3", a, P["up1"])
        u = torch.cat([upc("up1", c7, P["conv1.0"]), c1s], 1)
        a = conv("conv1.0", u, P["conv1.3"])
        c8 = conv("conv1.3", a, None)              # fp32 accumulators -> fused head
        hw = torch.from_numpy(np.asarray(sd["out_conv.weight"]))
        hb = torch.from_numpy(np.asarray(sd["out_conv.bias"]))
        if head is not None:
            c8, hw = rnd(c8, head), rnd(hw, head)
        return F.conv2d(c8, hw, hb)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=26)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--plans", nargs="+", default=["bf16", "fp16", "bf16_l0dec16"])
    ap.add_argument("--weights", default="pretrained")
    ap.add_argument("--head", nargs="+", default=["fp32"], help="head operand types to emulate (fp32 fp16 bf16)")
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 1)
    sys.path.insert(0, REPO)
    from bench import gen_pages
    sd = syn.make_state_dict(0, 3, 3, a.weights)
    x = torch.from_numpy(gen_pages(1000, a.images, a.size, 3))
    refs = []
    t0 = time.time()
    for i in range(a.images):
        lg = orc.unet_forward(sd, x[i:i + 1]).numpy()[0]
        refs.append((lg, orc.masks_from_logits(lg)))
    print(f"oracle: {time.time() - t0:.1f}s", flush=True)
    for pn, hd in [(p, h) for p in a.plans for h in a.head]:
        plan = plan_of(pn)
        ious, errs, worst = [], [], None
        for i in range(a.images):
            lg = emulate(sd, x[i:i + 1], plan, None if hd == "fp32" else hd).numpy()[0]
            m = orc.masks_from_logits(lg)
            errs.append(float(np.abs(lg - refs[i][0]).max()))
            for f in orc.FIELDS:
                iou = orc.mask_iou(m[f], refs[i][1][f])
                ious.append(iou)
                if worst is None or iou < worst[0]:
                    worst = (iou, i, f, int((m[f] != refs[i][1][f]).sum()), int(refs[i][1][f].sum()))
        print(f"{pn + ' head ' + hd:24s} IoU min {min(ious):.5f} mean {np.mean(ious):.5f}  max|dlogit| {max(errs):.3e}  "
              f"worst (iou, image, field, diff px, ref px) {worst}", flush=True)


if __name__ == "__main__":
    main()
