"""The C-ABI library builds, loads and exports every symbol include/unet_mi355x.h declares.
CPU-only: no compute call is made without a GPU."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "unet_mi355x.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(unet_[a-z_]+)\s*\(", src)))


def test_header_declares_abi():
    fns = declared_functions()
    for f in ("unet_create", "unet_load_weights", "unet_forward", "unet_destroy", "unet_last_error"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    from unet_mi355x import native
    lib = native.load_library()
    for f in declared_functions():
        assert hasattr(lib, f), f
        assert f in native.SIGNATURES, f
    assert lib.unet_abi_version() == native.ABI_VERSION == 5
    assert lib.unet_last_error() is not None


def test_create_rejects_bad_config_without_gpu():
    from unet_mi355x import native
    lib = native.load_library()
    h = ctypes.c_void_p()
    bad = native.UnetConfig(2, 3, 1, 0, (ctypes.c_float * 4)(0.25, 0.4, 0.3, 0.5))
    assert lib.unet_create(ctypes.byref(bad), ctypes.byref(h)) == native.UNET_EINVAL
    assert b"n_channels" in lib.unet_last_error()
    assert lib.unet_forward(None, None, 0, 0, None, None, 0, 1, 16, 16, None) == native.UNET_EINVAL


@pytest.mark.parametrize("thr", [0.25, 0.40, 0.30, 0.5, 1e-6, 0.999999])
def test_logit_cut_matches_fp32_sigmoid(thr):
    """Masks are thresholded as logit > cut (no exp on the device); around the cut and over
    a wide sweep the predicate must equal torch.sigmoid(x) > thr (inference.py:72-78) for
    every fp32 value, up to the last-ulp disagreement of the two sigmoid implementations."""
    import numpy as np
    import torch
    from unet_mi355x import native
    lib = native.load_library()
    cut = np.float32(lib.unet_logit_cut(thr))
    assert abs(float(cut) - np.log(thr / (1 - thr))) < 1e-3 * max(1.0, abs(np.log(thr / (1 - thr))))
    # every float within 4096 ulps of the cut, plus a wide log sweep of both signs
    bits = cut.view(np.int32).astype(np.int64) + np.arange(-4096, 4097)
    near = bits.astype(np.int32).view(np.float32)
    sweep = np.concatenate([np.geomspace(1e-8, 80, 20001), -np.geomspace(1e-8, 80, 20001)]).astype(np.float32)
    x = np.concatenate([near, sweep])
    ours = x > cut
    # fp32 sigmoids differ in the last ulp between libraries (glibc expf, numpy's SIMD exp,
    # torch's Sleef); each may move the boundary by a hair (up to ~3e-8 in the flat
    # region around thr=0.5) and nowhere else.
    for sig in (lambda v: np.float32(1) / (np.float32(1) + np.exp(-v)),
                lambda v: torch.sigmoid(torch.from_numpy(v)).numpy()):
        diff = ours != (sig(x) > np.float32(thr))
        assert np.all(np.abs(x[diff] - cut) <= 1e-6 * max(1.0, abs(float(cut)))), x[diff]

def test_logit_cut_degenerate_thresholds():
    import math
    from unet_mi355x import native
    lib = native.load_library()
    assert lib.unet_logit_cut(1.0) == math.inf
    assert lib.unet_logit_cut(-0.5) == -math.inf


def test_rccl_unique_id_without_gpu():
    """The multi-GPU C-ABI extras load RCCL at run time (dlopen); the bootstrap id of rank 0 is
    produced without a GPU (the all-gather itself is a -m gpu test)."""
    from unet_mi355x import native
    uid = native.Handle.comm_unique_id()
    assert len(uid) == native.COMM_ID_BYTES and any(uid)
