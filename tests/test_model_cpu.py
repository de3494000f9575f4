"""Drop-in module surface on CPU: constructor, state_dict keys, strict loading, and the
loud failure (no CPU fallback) of forward."""
import numpy as np
import pytest
import torch

from unet_mi355x import synthetic as syn
from unet_mi355x.model import UNet
import unet_model  # the drop-in shim module


def test_state_dict_keys_and_shapes_match_reference_layout():
    m = UNet(3, 3)
    sd = m.state_dict()
    ref = syn.unet_shapes(3, 3)
    assert list(sd.keys()) == [k for k, _ in ref]
    for k, shape in ref:
        assert tuple(sd[k].shape) == tuple(shape), k
    assert float(m.out_conv.bias.detach()[0]) == -4.0            # unet_model.py:53
    assert unet_model.UNet is UNet


def test_strict_load_of_synthetic_state_dict():
    m = UNet(1, 3)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(3, 1, 3).items()}
    m.load_state_dict(sd, strict=True)
    bad = dict(sd)
    bad.pop("up1.bias")
    with pytest.raises(RuntimeError):
        m.load_state_dict(bad, strict=True)


def test_forward_on_cpu_fails_loudly():
    m = UNet(3, 3).eval()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 3, 32, 32))
    with pytest.raises(RuntimeError, match="divisible by 16"):
        m(torch.zeros(1, 3, 40, 32))


def test_bad_dtype_rejected():
    with pytest.raises(ValueError):
        UNet(3, 3, compute_dtype="int8")
