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
    assert lib.unet_abi_version() == 1
    assert lib.unet_last_error() is not None


def test_create_rejects_bad_config_without_gpu():
    from unet_mi355x import native
    lib = native.load_library()
    h = ctypes.c_void_p()
    bad = native.UnetConfig(2, 3, 1, 0, (ctypes.c_float * 4)(0.25, 0.4, 0.3, 0.5))
    assert lib.unet_create(ctypes.byref(bad), ctypes.byref(h)) == native.UNET_EINVAL
    assert b"n_channels" in lib.unet_last_error()
    assert lib.unet_forward(None, None, 0, 0, None, None, 0, 1, 16, 16, None) == native.UNET_EINVAL
