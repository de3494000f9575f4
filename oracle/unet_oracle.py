"""CPU oracle for the UNet forward path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product path
(``unet_mi355x``) never imports it and has no CPU fallback.

This is a restatement of the reference algorithm with the same PyTorch eager
aten ops the reference dispatches (conv2d, eval batch_norm, relu, max_pool2d,
conv_transpose2d, cat), written against a plain state_dict so it needs no
reference import.  Parity is pinned by ``tests/golden/*.npz``, generated in the
survey container by importing the reference itself
(``tests/golden/make_golden.py``): ``tests/test_oracle_golden.py`` checks this
restatement against every one of them.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5            # nn.BatchNorm2d default, unet_model.py:11,15
FIELDS = ["invoice_no", "date", "total_amount"]      # inference.py:12
THRESHOLDS = {"invoice_no": 0.25, "date": 0.40, "total_amount": 0.30}  # inference.py:76-78
IMG_SIZE = 512           # inference.py:10


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))


def double_conv(sd, name: str, x: torch.Tensor) -> torch.Tensor:
    """DoubleConv.forward, unet_model.py:9-20: (conv3x3 pad1 -> BN(eval) -> ReLU) x2."""
    for conv, bn in ((0, 1), (3, 4)):
        x = F.conv2d(x, _t(sd, f"{name}.net.{conv}.weight"), _t(sd, f"{name}.net.{conv}.bias"), padding=1)
        x = F.batch_norm(x, _t(sd, f"{name}.net.{bn}.running_mean"), _t(sd, f"{name}.net.{bn}.running_var"),
                         _t(sd, f"{name}.net.{bn}.weight"), _t(sd, f"{name}.net.{bn}.bias"),
                         training=False, eps=BN_EPS)
        x = F.relu(x)
    return x


def up(sd, name: str, x: torch.Tensor) -> torch.Tensor:
    """nn.ConvTranspose2d(Cin, Cout, 2, stride=2), unet_model.py:38,41,44,47."""
    return F.conv_transpose2d(x, _t(sd, f"{name}.weight"), _t(sd, f"{name}.bias"), stride=2)


def unet_forward(sd, x: torch.Tensor, return_intermediates: bool = False):
    """UNet.forward, unet_model.py:55-86 (fp32, NCHW, CPU)."""
    x = x.float()
    if x.shape[-1] % 16 or x.shape[-2] % 16:
        # the reference fails inside torch.cat; mirror the error class
        raise RuntimeError("UNet forward needs H and W divisible by 16")
    with torch.no_grad():
        c1 = double_conv(sd, "down1", x)              # :56
        p1 = F.max_pool2d(c1, 2)                      # :57 (MaxPool2d(2), :34)
        c2 = double_conv(sd, "down2", p1)             # :59
        p2 = F.max_pool2d(c2, 2)
        c3 = double_conv(sd, "down3", p2)             # :62
        p3 = F.max_pool2d(c3, 2)
        c4 = double_conv(sd, "down4", p3)             # :65
        p4 = F.max_pool2d(c4, 2)
        bn = double_conv(sd, "bottleneck", p4)        # :68
        u4 = torch.cat([up(sd, "up4", bn), c4], 1)    # :70-71, upsampled first
        c5 = double_conv(sd, "conv4", u4)             # :72
        u3 = torch.cat([up(sd, "up3", c5), c3], 1)    # :74-75
        c6 = double_conv(sd, "conv3", u3)
        u2 = torch.cat([up(sd, "up2", c6), c2], 1)    # :78-79
        c7 = double_conv(sd, "conv2", u2)
        u1 = torch.cat([up(sd, "up1", c7), c1], 1)    # :82-83
        c8 = double_conv(sd, "conv1", u1)
        out = F.conv2d(c8, _t(sd, "out_conv.weight"), _t(sd, "out_conv.bias"))  # :86
    if return_intermediates:
        return out, dict(c1=c1, p1=p1, c2=c2, p2=p2, c3=c3, p3=p3, c4=c4, p4=p4, bn=bn,
                         c5=c5, c6=c6, c7=c7, c8=c8)
    return out


def masks_from_logits(logits: np.ndarray) -> dict:
    """inference.py:72-79: sigmoid in fp32, then strict '>' against the fp32 constants."""
    prob = torch.sigmoid(torch.from_numpy(np.ascontiguousarray(logits, dtype=np.float32))).numpy()
    return {k: prob[i] > np.float32(THRESHOLDS[k]) for i, k in enumerate(FIELDS)}


def crop_boxes(masks: dict, ow: int, oh: int) -> dict:
    """inference.py:84-121: bbox of each mask, scaled to the original size, 15% pad, clamp.

    Returns key -> (x1, y1, x2, y2) or None (empty mask or degenerate box).  The
    mean<3 rejection (inference.py:123-125) needs the pixels and is applied by
    the caller that holds the image.
    """
    out = {}
    for key, mask in masks.items():
        ys, xs = np.where(mask)
        if len(xs) == 0 or len(ys) == 0:
            out[key] = None
            continue
        mx1, mx2 = xs.min(), xs.max()
        my1, my2 = ys.min(), ys.max()
        sx, sy = ow / IMG_SIZE, oh / IMG_SIZE
        x1, x2, y1, y2 = int(mx1 * sx), int(mx2 * sx), int(my1 * sy), int(my2 * sy)
        px, py = int((x2 - x1) * 0.15), int((y2 - y1) * 0.15)
        x1, y1 = max(0, x1 - px), max(0, y1 - py)
        x2, y2 = min(ow, x2 + px), min(oh, y2 + py)
        out[key] = None if (x2 <= x1 or y2 <= y1) else (x1, y1, x2, y2)
    return out


def mask_iou(a: np.ndarray, b: np.ndarray) -> float:
    """Intersection over union of two boolean masks; 1.0 when both are empty."""
    a = a.astype(bool)
    b = b.astype(bool)
    union = np.logical_or(a, b).sum()
    if union == 0:
        return 1.0
    return float(np.logical_and(a, b).sum() / union)


# ---- run_unet restated on the CPU (inference.py:17-129): the CPU baseline's end-to-end leg ----

def load_model_state(checkpoint_path: str):
    """inference.py:17-24 on the CPU: build the UNet(3, 3) module tree (parameter allocation and
    default init, as ``UNet(3, 3)`` does), torch.load the checkpoint, strict load_state_dict,
    eval; returns the loaded state_dict the functional forward reads."""
    from unet_mi355x.model import UNet as _ModuleTree   # the reference's module tree, parameters only
    model = _ModuleTree(3, 3)
    state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    model.load_state_dict(state)
    model.eval()
    return {k: v.detach() for k, v in model.state_dict().items()}


def preprocess(pil_img) -> torch.Tensor:
    """inference.py:30-44: RGB, /255 in float32, HWC -> CHW, batch of 1."""
    arr = np.array(pil_img.convert("RGB")).astype(np.float32) / 255.0
    if arr.ndim != 3 or arr.shape[2] != 3:
        raise ValueError(f"Invalid image shape: {arr.shape}")
    return torch.from_numpy(arr.transpose(2, 0, 1)).unsqueeze(0)


def run_unet(pil_img, checkpoint_path: str):
    """inference.py:50-129: load the model (every call, :58), resize to 512 with PIL's default
    filter (:63), forward, sigmoid + thresholds (:72-79), bbox -> 15 % pad -> crop, rejecting
    empty / degenerate / near-black crops (:84-127).  Returns (masks, crops)."""
    sd = load_model_state(checkpoint_path)
    ow, oh = pil_img.size
    x = preprocess(pil_img.resize((IMG_SIZE, IMG_SIZE)))
    logits = unet_forward(sd, x).numpy()[0]
    masks = masks_from_logits(logits)
    crops = {}
    for key, box in crop_boxes(masks, ow, oh).items():
        crop = None if box is None else pil_img.crop(box)
        if crop is not None:
            arr = np.array(crop)
            if arr.size == 0 or arr.mean() < 3:
                crop = None
        crops[key] = crop
    return masks, crops
