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


def test_training_mode_raises_clearly():
    """the drop-in is inference-only; training-mode use with grad enabled raises at the
    call instead of returning eval-mode outputs without a graph (reference train.py imports UNet)."""
    m = UNet(3, 3)
    assert m.training
    with pytest.raises(RuntimeError, match="inference-only"):
        m(torch.zeros(1, 3, 32, 32))


def test_bad_dtype_rejected():
    with pytest.raises(ValueError):
        UNet(3, 3, compute_dtype="int8")


def _np_box(mask):
    ys, xs = np.where(mask)
    return None if len(xs) == 0 else (xs.min(), ys.min(), xs.max(), ys.max())


def test_crops_from_boxes_equal_crops_from_masks():
    """run_unet's crop step from device boxes (x0, y0, x1, y1 / -1s) == the reference's
    np.where path (inference.py:84-127) on the same masks, incl. empty / 1-pixel masks."""
    from PIL import Image
    from unet_mi355x import inference as inf
    rng = np.random.default_rng(0)
    img = Image.fromarray(rng.integers(0, 256, (400, 600, 3), dtype=np.uint8), mode="RGB")
    dark = Image.fromarray(np.zeros((300, 200, 3), dtype=np.uint8), mode="RGB")
    for trial in range(20):
        masks = {}
        for i, k in enumerate(inf.FIELDS):
            m = np.zeros((512, 512), dtype=bool)
            kind = (trial + i) % 4
            if kind == 1:
                m[rng.integers(0, 512), rng.integers(0, 512)] = True
            elif kind >= 2:
                y0, x0 = rng.integers(0, 400, 2)
                m[y0:y0 + rng.integers(1, 100), x0:x0 + rng.integers(1, 100)] = rng.random() < 0.9
            masks[k] = m
        boxes = np.array([_np_box(masks[k]) or (-1, -1, -1, -1) for k in inf.FIELDS], dtype=np.int32)
        for pil in (img, dark):
            a = inf.masks_to_crops(pil, masks)
            b = inf.boxes_to_crops(pil, boxes)
            for k in inf.FIELDS:
                assert (a[k] is None) == (b[k] is None), (trial, k)
                if a[k] is not None:
                    assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]))
