"""Portable synthetic data for the UNet forward path.

The reference's trained checkpoint (``checkpoints/best_unet_model.pth``) is a
Git-LFS pointer only, so every weight set used here is
generated.  To keep golden fixtures valid on any host and any torch version the
generator does not use torch's RNG: it is a counter-based splitmix64 stream per
(seed, tensor name), mapped to uniforms (53-bit) and to normals (Box-Muller).

State-dict layout (136 keys, registration order) follows
``unet_model.py:24-53`` (reference): nine ``DoubleConv`` blocks
(``unet_model.py:6-20``: ``net.0`` conv3x3, ``net.1`` BN, ``net.3`` conv3x3,
``net.4`` BN), four ``ConvTranspose2d(k=2, s=2)`` ups and the 1x1 ``out_conv``.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# (block name, in_ch, out_ch) in registration order, unet_model.py:29-50.
DOUBLE_CONVS = ("down1", "down2", "down3", "down4", "bottleneck",
                "conv4", "conv3", "conv2", "conv1")
UPS = ("up4", "up3", "up2", "up1")
PRETRAINED_DELTA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "pretrained_delta.npz")


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _stream_base(seed: int, key: str) -> np.uint64:
    base = (_fnv1a64(key) ^ ((seed * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF))
    # one extra mixing round so nearby seeds give unrelated streams
    return _splitmix64(np.array([base], dtype=np.uint64))[0]


def uniform(seed: int, key: str, n: int, offset: int = 0) -> np.ndarray:
    """n float64 uniforms in [0, 1) from stream (seed, key), counters offset..offset+n."""
    ctr = np.arange(offset, offset + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = _splitmix64(ctr + _stream_base(seed, key))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed: int, key: str, n: int) -> np.ndarray:
    """n float64 standard normals (Box-Muller on counter pairs)."""
    m = (n + 1) // 2
    u = uniform(seed, key, 2 * m)
    u1, u2 = u[0::2], u[1::2]
    r = np.sqrt(-2.0 * np.log1p(-u1))
    t = 2.0 * math.pi * u2
    out = np.empty(2 * m, dtype=np.float64)
    out[0::2] = r * np.cos(t)
    out[1::2] = r * np.sin(t)
    return out[:n]


def unet_shapes(n_channels: int = 3, n_classes: int = 3, base: int = 64):
    """Ordered (key, shape) list of the reference UNet state_dict (unet_model.py:24-53)."""
    c = [base, base * 2, base * 4, base * 8, base * 16]
    dc = {
        "down1": (n_channels, c[0]), "down2": (c[0], c[1]), "down3": (c[1], c[2]),
        "down4": (c[2], c[3]), "bottleneck": (c[3], c[4]),
        "conv4": (c[4], c[3]), "conv3": (c[3], c[2]), "conv2": (c[2], c[1]),
        "conv1": (c[1], c[0]),
    }
    up = {"up4": (c[4], c[3]), "up3": (c[3], c[2]), "up2": (c[2], c[1]), "up1": (c[1], c[0])}
    order = ["down1", "down2", "down3", "down4", "bottleneck",
             "up4", "conv4", "up3", "conv3", "up2", "conv2", "up1", "conv1"]
    out = []
    for name in order:
        if name in dc:
            ci, co = dc[name]
            for idx, cin in ((0, ci), (3, co)):
                out.append((f"{name}.net.{idx}.weight", (co, cin, 3, 3)))
                out.append((f"{name}.net.{idx}.bias", (co,)))
                bn = idx + 1
                out.append((f"{name}.net.{bn}.weight", (co,)))
                out.append((f"{name}.net.{bn}.bias", (co,)))
                out.append((f"{name}.net.{bn}.running_mean", (co,)))
                out.append((f"{name}.net.{bn}.running_var", (co,)))
                out.append((f"{name}.net.{bn}.num_batches_tracked", ()))
        else:
            ci, co = up[name]
            out.append((f"{name}.weight", (ci, co, 2, 2)))
            out.append((f"{name}.bias", (co,)))
    out.append(("out_conv.weight", (n_classes, c[0], 1, 1)))
    out.append(("out_conv.bias", (n_classes,)))
    return out


def _fan_in(key: str, shape) -> int:
    if key.startswith("up"):
        # ConvTranspose2d weight (Cin, Cout, kh, kw): every output sums over Cin taps.
        return int(shape[0])
    return int(np.prod(shape[1:]))


def make_state_dict(seed: int = 0, n_channels: int = 3, n_classes: int = 3,
                    profile: str = "structured", out_bias: float | None = None,
                    base: int = 64) -> "OrderedDict[str, np.ndarray]":
    """Deterministic UNet state_dict (numpy; fp32 tensors, int64 num_batches_tracked).

    profile "torch_default": the reference constructor's own init semantics
      (kaiming-uniform a=sqrt(5) bounds 1/sqrt(fan_in), identity BN, out bias -4
      as unet_model.py:52-53) -- logits sit near -4, every mask is empty.
    profile "structured": He-normal conv weights, randomised eval BN statistics,
      so activations stay O(1) through all 19 layers and masks are non-trivial.
    profile "pretrained": the seed-0 structured weights with the ~13 k BatchNorm-affine /
      ConvTranspose-bias / out_conv parameters replaced by the values fine-tuned on the
      synthetic invoice fields (tools/pretrain_synthetic.py, data/pretrained_delta.npz):
      a trained-like, bimodal logit distribution for mask-IoU measurements.
    """
    if profile == "pretrained":
        if seed != 0 or n_classes != 3 or base != 64:
            raise ValueError("profile 'pretrained' exists for seed 0, n_classes 3, base 64 only")
        sd = make_state_dict(0, n_channels, 3, "structured", None, 64)
        z = np.load(PRETRAINED_DELTA)
        if n_channels == 3 and bytes(z["__base_checksum__"]).decode() != state_dict_checksum(sd):
            raise RuntimeError("pretrained delta was made for different base weights")
        for k in z.files:
            if k.startswith("__"):
                continue
            if sd[k].shape != z[k].shape:
                raise RuntimeError(f"pretrained delta: shape mismatch for {k}")
            sd[k] = np.asarray(z[k], dtype=np.float32)
        if out_bias is not None:
            sd["out_conv.bias"] = np.full(n_classes, float(out_bias), dtype=np.float32)
        return sd
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape in unet_shapes(n_channels, n_classes, base):
        n = int(np.prod(shape)) if shape else 1
        if key.endswith("num_batches_tracked"):
            sd[key] = np.array(0 if profile == "torch_default" else 1000, dtype=np.int64)
            continue
        is_bn = ".net.1." in key or ".net.4." in key
        if profile == "torch_default":
            if is_bn:
                v = {"weight": 1.0, "bias": 0.0, "running_mean": 0.0, "running_var": 1.0}[key.rsplit(".", 1)[1]]
                arr = np.full(n, v)
            else:
                wkey = key[:-len("bias")] + "weight" if key.endswith("bias") else key
                wshape = dict(unet_shapes(n_channels, n_classes, base))[wkey]
                fan = _fan_in(wkey, wshape) if not wkey.startswith("up") else int(np.prod(wshape[1:]))
                bound = 1.0 / math.sqrt(fan)
                arr = (uniform(seed, key, n) * 2.0 - 1.0) * bound
                if key == "out_conv.bias":
                    arr = np.full(n, -4.0)
        else:
            leaf = key.rsplit(".", 1)[1]
            if is_bn:
                if leaf == "weight":
                    arr = 0.8 + 0.4 * uniform(seed, key, n)
                elif leaf == "bias":
                    arr = 0.1 * normal(seed, key, n)
                elif leaf == "running_mean":
                    arr = 0.1 * normal(seed, key, n)
                else:
                    arr = 0.5 + uniform(seed, key, n)
            elif leaf == "weight":
                std = math.sqrt((1.0 if key.startswith("out_conv") else 2.0) / _fan_in(key, shape))
                arr = std * normal(seed, key, n)
            else:
                arr = 0.02 * normal(seed, key, n)
                if key == "out_conv.bias":
                    arr = np.full(n, 0.0 if out_bias is None else out_bias)
        if key == "out_conv.bias" and out_bias is not None:
            arr = np.full(n, float(out_bias))
        sd[key] = np.asarray(arr, dtype=np.float32).reshape(shape)
    return sd


def state_dict_checksum(sd) -> str:
    """sha256 over the raw little-endian bytes of every tensor in order (fixture drift guard)."""
    import hashlib
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


def uniform_batch(seed: int, n: int, c: int, h: int, w: int) -> np.ndarray:
    """U[0,1) fp32 NCHW batch (SURVEY.md §8d distribution 1)."""
    return uniform(seed, "input.uniform", n * c * h * w).astype(np.float32).reshape(n, c, h, w)


def _page_rects(seed: int, i: int, h: int, w: int, rects_per_512sq: int):
    """Background level and the (y0, x0, rh, rw, value) rectangles of page i."""
    key = f"page.{i}"
    sy, sx = h / 512.0, w / 512.0
    nrect = max(1, int(round(rects_per_512sq * h * w / (512.0 * 512.0))))
    bg = 0.8 + 0.2 * uniform(seed, key + ".bg", 1)[0]
    r = uniform(seed, key + ".rects", nrect * 5).reshape(nrect, 5)
    rects = []
    for k in range(nrect):
        rh = max(1, int((6 + 34 * r[k, 0]) * sy))
        rw = max(1, int((20 + 180 * r[k, 1]) * sx))
        y0 = int(r[k, 2] * max(1, h - rh))
        x0 = int(r[k, 3] * max(1, w - rw))
        rects.append((y0, x0, rh, rw, 0.3 * r[k, 4]))
    return bg, rects


def invoice_pages(seed: int, n: int, h: int = 512, w: int = 512, channels: int = 3,
                  rects_per_512sq: int = 40) -> np.ndarray:
    """Invoice-like gray pages, fp32 NCHW in [0,1] (SURVEY.md §8d distribution 2).

    White-ish background U[0.8,1], dark text-like rectangles (h in [6,40),
    w in [20,200) per 512 px, value U[0,0.3]), N(0,0.02) noise, clipped.
    Gray is replicated over ``channels`` exactly as PIL ``convert("RGB")`` does
    for a grayscale photo (inference.py:35).
    """
    out = np.empty((n, 1, h, w), dtype=np.float32)
    for i in range(n):
        bg, rects = _page_rects(seed, i, h, w, rects_per_512sq)
        page = np.full((h, w), bg, dtype=np.float64)
        for y0, x0, rh, rw, v in rects:
            page[y0:y0 + rh, x0:x0 + rw] = v
        page += 0.02 * normal(seed, f"page.{i}.noise", h * w).reshape(h, w)
        out[i, 0] = np.clip(page, 0.0, 1.0)
    if channels == 1:
        return out
    return np.ascontiguousarray(np.repeat(out, channels, axis=1))


def invoice_fields(seed: int, n: int, h: int = 512, w: int = 512,
                   rects_per_512sq: int = 40) -> np.ndarray:
    """Synthetic field masks [n, 3, h, w] (uint8) for the pages of ``invoice_pages``.

    A stand-in for the three trained fields (``inference.py:12``: invoice_no, date,
    total_amount), defined by rectangle geometry so that a segmentation net can learn them:
    field 0 = tall rectangles (height >= 20 px per 512), field 1 = wide ones (width >= 110),
    field 2 = the darkest ones (value < 0.15).  Later rectangles overwrite earlier ones,
    as on the page.  Used only to give the synthetic weights a trained-like (bimodal)
    logit distribution (tools/pretrain_synthetic.py).
    """
    out = np.zeros((n, 3, h, w), dtype=np.uint8)
    sy, sx = h / 512.0, w / 512.0
    for i in range(n):
        _, rects = _page_rects(seed, i, h, w, rects_per_512sq)
        for y0, x0, rh, rw, v in rects:
            out[i, :, y0:y0 + rh, x0:x0 + rw] = np.array(
                [rh >= 20 * sy, rw >= 110 * sx, v < 0.15], dtype=np.uint8)[:, None, None]
    return out
