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


def _reference_crops(pil, masks):
    """inference.py:84-127 through the oracle's restatement (oracle.crop_boxes + near-black rule)."""
    from oracle import unet_oracle as orc
    out = {}
    for k, box in orc.crop_boxes(masks, *pil.size).items():
        crop = None if box is None else pil.crop(box)
        if crop is not None:
            arr = np.array(crop)
            if arr.size == 0 or arr.mean() < 3:
                crop = None
        out[k] = crop
    return out


def test_crops_from_boxes_and_stats_equal_reference_crops():
    """run_unet's crop step -- from device boxes (crop_from_box), and from device crop statistics
    (crop_from_stats: rectangle + pixel sum, the near-black test as sum < 3 * count) -- equals the
    reference's np.where path (inference.py:84-127) on the same masks: empty / 1-pixel masks,
    random and dim photos (crop means around 3), RGB and L."""
    from PIL import Image
    from unet_mi355x import inference as inf
    rng = np.random.default_rng(0)
    photos = [Image.fromarray(rng.integers(0, 256, (400, 600, 3), dtype=np.uint8), mode="RGB"),
              Image.fromarray(np.zeros((300, 200, 3), dtype=np.uint8), mode="RGB"),
              Image.fromarray(rng.integers(0, 7, (333, 517, 3), dtype=np.uint8), mode="RGB"),
              Image.fromarray(rng.integers(0, 7, (500, 280), dtype=np.uint8), mode="L")]
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
        for pil in photos:
            a = _reference_crops(pil, masks)
            b = inf.boxes_to_crops(pil, boxes)
            arr = np.asarray(pil)
            ch = 3 if arr.ndim == 3 else 1
            c = {}
            for i, k in enumerate(inf.FIELDS):
                r = (-1, -1, -1, -1) if boxes[i, 2] < 0 else inf.crop_rect(boxes[i], *pil.size)
                s = 0 if r[2] < 0 else int(arr[r[1]:r[3], r[0]:r[2]].astype(np.int64).sum())
                c[k] = inf.crop_from_stats(pil, r, s, ch)
            for k in inf.FIELDS:
                assert (a[k] is None) == (b[k] is None) == (c[k] is None), (trial, k, pil.mode)
                if a[k] is not None:
                    assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]))
                    assert np.array_equal(np.asarray(a[k]), np.asarray(c[k]))


def test_photo_array_equals_numpy_view_of_the_photo():
    """run_unet's one-pass photo packing (inference.photo_array) == np.asarray(photo), the bytes the
    reference's preprocess reads (inference.py:30-44): RGB and L, odd sizes, a 1x1 and a 12 MP photo;
    other modes go through np.asarray unchanged."""
    from PIL import Image
    from unet_mi355x.inference import photo_array
    rng = np.random.default_rng(11)
    for shape, mode in [((400, 600, 3), "RGB"), ((401, 599, 3), "RGB"), ((37, 23), "L"), ((1, 1, 3), "RGB"),
                        ((3024, 4032, 3), "RGB")]:
        pil = Image.fromarray(rng.integers(0, 256, shape, dtype=np.uint8), mode)
        got = photo_array(pil)
        assert got.dtype == np.uint8 and got.shape == shape and np.array_equal(got, np.asarray(pil)), shape
    rgba = Image.fromarray(rng.integers(0, 256, (5, 7, 4), dtype=np.uint8), "RGBA")
    assert np.array_equal(photo_array(rgba), np.asarray(rgba))


def test_doubleconv_standalone_surface_on_cpu():
    """DoubleConv (unet_model.py:6-20) keeps the reference's 14 state_dict keys; called on its own it
    runs the native block path, so on CPU it fails loudly (no fallback), checks its channel count,
    and the library refuses block shapes the native kernels do not cover before touching a GPU."""
    import ctypes
    from unet_mi355x import native
    from unet_mi355x.model import DoubleConv
    d = DoubleConv(64, 128).eval()
    assert [k for k in d.state_dict()] == [f"net.{i}.{p}" for i, p in
                                           [(0, "weight"), (0, "bias"), (1, "weight"), (1, "bias"), (1, "running_mean"),
                                            (1, "running_var"), (1, "num_batches_tracked"), (3, "weight"), (3, "bias"),
                                            (4, "weight"), (4, "bias"), (4, "running_mean"), (4, "running_var"),
                                            (4, "num_batches_tracked")]]
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        d(torch.zeros(1, 64, 8, 8))
    with pytest.raises(RuntimeError, match="64 channels"):
        d(torch.zeros(1, 32, 8, 8))
    assert UNet(3, 3, compute_dtype="mixed").conv2.compute_dtype == "mixed"
    lib = native.load_library()
    b = ctypes.c_void_p()
    for cin, cout in ((5, 64), (3, 128), (64, 96)):
        rc = lib.unet_block_create(ctypes.byref(native.BlockConfig(cin, cout, 1, 0)), ctypes.byref(b))
        assert rc == native.UNET_ESHAPE and b"DoubleConv" in lib.unet_last_error(), (cin, cout)


def test_copy_rgbx_equals_the_photo_pixels():
    """run_unet's upload of an "RGB" photo (inference.copy_rgbx): Pillow's own RGBX pixels through its
    zero-copy Arrow export, whose R, G, B bytes equal np.asarray(photo) -- plain, odd-sized, 1 x 1, cropped
    and converted photos; None (the caller packs with photo_array) for other modes, a too small buffer and
    a photo Pillow keeps in several memory blocks."""
    from PIL import Image
    from unet_mi355x import inference as inf
    rng = np.random.default_rng(3)
    base = Image.fromarray(rng.integers(0, 256, (400, 600, 3), dtype=np.uint8))
    photos = [base, Image.fromarray(rng.integers(0, 256, (23, 37, 3), dtype=np.uint8)),
              Image.fromarray(rng.integers(0, 256, (1, 1, 3), dtype=np.uint8)), base.crop((13, 7, 301, 222)),
              Image.fromarray(rng.integers(0, 256, (50, 70, 4), dtype=np.uint8), "RGBA").convert("RGB"),
              base.convert("L").convert("RGB")]
    for p in photos:
        w, h = p.size
        buf = np.full(w * h * 4 + 64, 7, np.uint8)
        shape = inf.copy_rgbx(p, buf.ctypes.data, buf.size)
        if shape is None:   # the export is an optimisation: an older Pillow may not have it
            continue
        assert shape == (h, w, 4)
        px = buf[:w * h * 4].reshape(h, w, 4)
        assert np.array_equal(px[..., :3], np.asarray(p)), p.size
        assert (buf[w * h * 4:] == 7).all()
    small = np.empty(16, np.uint8)
    assert inf.copy_rgbx(base, small.ctypes.data, small.size) is None
    assert inf.copy_rgbx(base.convert("L"), small.ctypes.data, 1 << 30) is None
    assert inf.copy_rgbx(base.convert("RGBA"), small.ctypes.data, 1 << 30) is None
    big = Image.new("RGB", (4032, 3024))
    huge = np.empty(4032 * 3024 * 4, np.uint8)
    shape = inf.copy_rgbx(big, huge.ctypes.data, huge.size)
    assert shape is None or shape == (3024, 4032, 4)


def test_staging_outputs_are_one_block_in_copy_order():
    """run_unet's output buffers are carved from one block, masks | boxes | rects | sums, so the photo
    graph copies the three small ones back as one (unet_photo_graph_create merges adjacent copies; the
    masks copy is its own node, retargeted per call): each view contiguous, of the right dtype and shape,
    int64 sums 8-byte aligned, no gaps."""
    from unet_mi355x import inference as inf
    block = torch.empty(inf._Staging._out_bytes(), dtype=torch.uint8)
    m, b, r, s = inf._Staging._outputs(block)
    n = len(inf.FIELDS)
    assert m.shape == (1, n, 512, 512) and m.dtype == torch.uint8
    assert b.shape == (1, n, 4) and b.dtype == torch.int32
    assert r.shape == (n, 4) and r.dtype == torch.int32
    assert s.shape == (n,) and s.dtype == torch.int64
    base = block.data_ptr()
    ends = base
    for t in (m, b, r, s):
        assert t.is_contiguous() and t.data_ptr() == ends
        ends += t.numel() * t.element_size()
    assert ends == base + block.numel()
    assert (s.data_ptr() - base) % 8 == 0


def _plain_pool(monkeypatch, size=4):
    from unet_mi355x import inference as inf
    real_empty = torch.empty
    monkeypatch.setattr(torch, "empty", lambda *a, **k: real_empty(*a, **{x: v for x, v in k.items() if x != "pin_memory"}))
    return inf._MaskPool((3, 8, 8), size)


def test_mask_blocks_are_lent_until_the_last_view_dies(monkeypatch):
    """run_unet's pinned mask blocks (inference._MaskPool): a block is lent again only once no mask returned
    in it is alive (a weakref.finalize on the owner every view keeps alive hands it back); with every
    block lent, take() gives None (the copying path).  CPU stand-in: pinned allocation replaced by a plain
    one."""
    import gc
    from unet_mi355x import inference as inf
    pool = _plain_pool(monkeypatch)
    t0, a0 = pool.take()
    assert pool.blocks[0] is t0 and a0.dtype == np.bool_ and a0.shape == (3, 8, 8)
    held = {k: a0[j] for j, k in enumerate(inf.FIELDS)}
    del a0
    t1, a1 = pool.take()
    assert t1 is pool.blocks[1]                         # block 0 is held by the masks' views
    del a1
    assert pool.take()[0] is pool.blocks[1]             # block 1's views are gone: lent again (and dropped)
    one = held["date"]
    del held
    assert pool.take()[0] is pool.blocks[1]             # one field kept: block 0 still held
    del one
    gc.collect()
    assert pool.take()[0] is pool.blocks[0]             # all dropped: block 0 free again
    keep = [pool.take()[1][0] for _ in range(pool.size)]
    assert len(pool.blocks) == pool.size and pool.take() is None   # every block held: the copying path
    del keep
    assert pool.take() is not None
    # views survive a copy of the dict they came in and a numpy view of a view
    t, a = pool.take()
    v = a[2][1:, ::2]
    del a
    i = [b is t for b in pool.blocks].index(True)
    assert not pool.idle[i]
    del v
    assert pool.idle[i]


def test_mask_block_of_a_failed_call_goes_back(monkeypatch):
    """A call that fails after taking a block (its bool array never reaches a caller) returns the block."""
    pool = _plain_pool(monkeypatch, size=1)

    def failing_call():
        lent = pool.take()
        raise RuntimeError("launch failed")
    for _ in range(3):
        try:
            failing_call()
        except RuntimeError:
            pass
        assert pool.idle == [True]


def test_weight_tracking_is_scoped_to_the_unet_tree():
    """the re-pack signature's tensor list is invalidated by the UNet tree's own modules (tracked
    subclasses of the reference's layer classes), not by process-global torch hooks: importing the package
    installs none, a foreign module's registrations leave the epoch alone, and every way of replacing a
    tensor of the tree -- parameter / buffer assignment, a replaced sub-module, _apply on a leaf --
    changes the UNet's signature."""
    import torch.nn as nn
    import torch.nn.modules.module as mm
    from unet_mi355x import model as mdl
    for d in ("_global_parameter_registration_hooks", "_global_buffer_registration_hooks",
              "_global_module_registration_hooks"):
        assert not getattr(mm, d, {}), d
    m = mdl.UNet(3, 3)
    assert type(m.down1.net[0]).__name__ == "Conv2d" and isinstance(m.down1.net[0], nn.Conv2d)
    assert "Conv2d(3, 64, kernel_size=(3, 3)" in repr(m)
    assert len(m.state_dict()) == 136
    sig0 = m._signature()
    e0 = mdl._TREE_EPOCH[0]
    foreign = nn.Linear(3, 3)
    foreign.weight = nn.Parameter(torch.zeros(3, 3))
    foreign.register_buffer("b", torch.zeros(1))
    assert mdl._TREE_EPOCH[0] == e0                     # other modules of the process are not touched
    assert m._signature() == sig0
    m.down2.net[0].weight = nn.Parameter(torch.zeros_like(m.down2.net[0].weight))
    sig1 = m._signature()
    assert sig1 != sig0
    m.conv3.net[4].running_mean = torch.zeros(256)      # buffer assignment (no register_buffer call)
    sig2 = m._signature()
    assert sig2 != sig1
    m.out_conv.float()                                   # _apply on a leaf (no change of storage here)
    m.up2 = mdl.ConvTranspose2d(256, 128, 2, stride=2)   # a replaced sub-module
    sig3 = m._signature()
    assert sig3 != sig2
    with torch.no_grad():
        m.up2.bias.add_(1)                               # in-place update: _version
    assert m._signature() != sig3
    m.up1 = nn.ConvTranspose2d(128, 64, 2, stride=2)     # a plain module: the signature walks the live tree
    s4 = m._signature()
    m.up1.weight = nn.Parameter(torch.zeros_like(m.up1.weight))
    assert not m._sig_tracked and m._signature() != s4
