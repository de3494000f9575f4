"""CPU restatement of Pillow's 8-bit BICUBIC resize -- TEST INFRASTRUCTURE ONLY.

The reference resizes every photo with ``PIL.Image.resize((512, 512))`` (inference.py:63,
and again inside preprocess, inference.py:35), i.e. Pillow's default BICUBIC filter.  That
algorithm lives in a dependency (Pillow, pinned 10.2.0 by the reference's requirements.txt:11;
12.2.0 in this image), not in the reference: libImaging/Resample.c, ``precompute_coeffs`` +
``normalize_coeffs_8bpc`` + ``ImagingResampleHorizontal_8bpc`` / ``..Vertical_8bpc``.
Restated here from its published algorithm:

* per output index: center = (i + 0.5) * scale, filterscale = max(scale, 1), support =
  2 * filterscale, taps [int(center - support + 0.5), int(center + support + 0.5)) clamped to
  the input, weights bicubic(a = -0.5)((x - center + 0.5) / filterscale) normalised to sum 1,
  then fixed point with 22 fractional bits rounded half away from zero;
* horizontal pass first (only over the rows the vertical pass reads), 8-bit clipped
  intermediate, then the vertical pass; each sample = clip8((1 << 21) + sum(in * w) >> 22).

Pinned against the installed Pillow itself (tests/test_preprocess_cpu.py, bit-exact).  Used
only by tests as the checker of the device resampler (csrc/unet_preprocess.hip).
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def coeffs(in_size: int, out_size: int):
    """(bounds [out][2] = (xmin, taps), fixed-point weights [out][ksize]) as Resample.c."""
    in0, in1 = 0.0, float(in_size)
    scale = filterscale = (in1 - in0) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for w in k:
            ww += w
        for x in range(xmax):
            v = k[x] / ww if ww != 0.0 else k[x]
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(v):
    return np.clip(v >> PRECISION_BITS, 0, 255)


def _pass(a: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    a = np.moveaxis(a, axis, 0)
    out = np.empty((len(bounds),) + a.shape[1:], np.int64)
    for i, (lo, n) in enumerate(bounds):
        acc = np.full(a.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += a[lo + t] * kk[i, t]
        out[i] = _clip8(acc)
    return np.moveaxis(out, 0, axis)


def resize(arr: np.ndarray, ow: int, oh: int) -> np.ndarray:
    """uint8 [H, W] or [H, W, C] -> uint8 [oh, ow(, C)] == PIL Image.resize((ow, oh)) (BICUBIC)."""
    ih, iw = arr.shape[:2]
    a = arr.astype(np.int64)
    bh, kh = coeffs(iw, ow)
    bv, kv = coeffs(ih, oh)
    if ow != iw:
        y0, y1 = (int(bv[0, 0]), int(bv[-1, 0] + bv[-1, 1])) if oh != ih else (0, ih)
        a = _pass(a[y0:y1], bh, kh, 1)
        bv = bv.copy()
        bv[:, 0] -= y0
    if oh != ih:
        a = _pass(a, bv, kv, 0)
    return a.astype(np.uint8)


def to_input(arr: np.ndarray, size: int = 512) -> np.ndarray:
    """inference.py:62-64 + :30-44 on a uint8 RGB/L array: resize, gray->RGB, /255 fp32, CHW."""
    r = resize(arr, size, size)
    if r.ndim == 2:
        r = np.repeat(r[..., None], 3, axis=2)
    return (r.astype(np.float32) / np.float32(255.0)).transpose(2, 0, 1)
