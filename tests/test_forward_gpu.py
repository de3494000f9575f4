"""Parity of the native MI355X forward (through the C-ABI) against the golden vectors the
reference produced and against the CPU oracle.  Needs a GPU: run with -m gpu.

Tolerances (max |err| / max(1, max|ref|)):
  fp32 path (exact-fp32 MFMA, different summation order)  <= 1e-4
  fp16 path (fp16 storage, fp32 accumulate)                <= 1.5e-2
  bf16 path (bf16 storage, fp32 accumulate)                <= 8e-2
Masks (fp32 path) must match the oracle to IoU >= 0.999 (north_star); 16-bit IoUs are
reported and bounded below.
"""
import glob
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import unet_oracle as orc
from unet_mi355x import synthetic as syn
from unet_mi355x.model import UNet

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = {"fp32": 1e-4, "fp16": 1.5e-2, "bf16": 8e-2}
DEV = "cuda:0"


def make_model(sd_np, c, dtype):
    m = UNet(c, 3, compute_dtype=dtype)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd_np.items()})
    return m.to(DEV).eval()


def rel_err(out, ref):
    return float(np.abs(out - ref).max()) / max(1.0, float(np.abs(ref).max()))


@pytest.mark.parametrize("dtype", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "unet_*.npz"))), ids=os.path.basename)
def test_golden_logits(path, dtype):
    z = np.load(path)
    c = int(z["n_channels"])
    sd = syn.make_state_dict(int(z["seed"]), c, 3, profile=str(z["profile"]))
    m = make_model(sd, c, dtype)
    with torch.no_grad():
        out = m(torch.from_numpy(z["x"]).to(DEV)).cpu().numpy()
    err = rel_err(out, z["logits"])
    print(f"{os.path.basename(path)} {dtype}: rel err {err:.3e}")
    assert out.shape == z["logits"].shape
    assert np.isfinite(out).all()
    assert err <= TOL[dtype]
    m.close()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_golden_intermediates(dtype):
    """Per-layer localisation: skips, pools, bottleneck and up-convs vs the reference hooks."""
    z = np.load(os.path.join(GOLD, "unet_c3_h16w16_n3_structured.npz"))
    sd = syn.make_state_dict(int(z["seed"]), 3, 3, profile=str(z["profile"]))
    m = make_model(sd, 3, dtype)
    x = torch.from_numpy(z["x"]).to(DEV)
    with torch.no_grad():
        m(x)
    torch.cuda.synchronize()
    for name, key in (("c1", "inter_c1"), ("c2", "inter_c2"), ("c3", "inter_c3"), ("c4", "inter_c4"),
                      ("bn", "inter_bn"), ("u1", "inter_u1_up"), ("u4", "inter_u4_up"), ("c7", "inter_c7")):
        ref = z[key]
        got = m.intermediate(name).cpu().numpy().reshape(ref.shape)
        err = rel_err(got, ref)
        print(f"{name} {dtype}: rel err {err:.3e}")
        assert err <= TOL[dtype], name
    m.close()


@pytest.mark.parametrize("c,n,h,w", [(3, 2, 64, 128), (1, 3, 96, 32), (3, 1, 160, 48)])
def test_fp32_vs_oracle_odd_shapes(c, n, h, w):
    sd = syn.make_state_dict(100 + h, c, 3, profile="structured")
    x = syn.uniform_batch(5 + w, n, c, h, w)
    ref = orc.unet_forward(sd, torch.from_numpy(x)).numpy()
    m = make_model(sd, c, "fp32")
    with torch.no_grad():
        out = m(torch.from_numpy(x).to(DEV)).cpu().numpy()
    err = rel_err(out, ref)
    print(f"fp32 {c}x{h}x{w} n={n}: rel err {err:.3e}")
    assert err <= TOL["fp32"]
    m.close()


def _recentred(seed, x, c=3):
    """Structured weights with out_conv bias shifted so ~10% of pixels pass each threshold."""
    sd = syn.make_state_dict(seed, c, 3, profile="structured")
    logits = orc.unet_forward(sd, torch.from_numpy(x)).numpy()
    thr = np.array([0.25, 0.40, 0.30])
    q = np.quantile(logits.transpose(1, 0, 2, 3).reshape(3, -1), 0.9, axis=1)
    sd["out_conv.bias"] = (sd["out_conv.bias"] + (np.log(thr / (1 - thr)) - q)).astype(np.float32)
    return sd, orc.unet_forward(sd, torch.from_numpy(x)).numpy()


def test_masks_512_all_dtypes():
    """Full-size 512x512 pages: fused masks (u8 and bit-packed) vs the oracle's masks."""
    x = syn.invoice_pages(21, 2, 512, 512, 3)
    sd, ref_logits = _recentred(21, x)
    ref_masks = np.stack([np.stack(list(orc.masks_from_logits(ref_logits[i]).values())) for i in range(2)])
    xd = torch.from_numpy(x).to(DEV)
    for dtype, min_iou in (("fp32", 0.999), ("fp16", 0.99), ("bf16", 0.95)):
        m = make_model(sd, 3, dtype)
        with torch.no_grad():
            masks, logits = m.forward_masks(xd, with_logits=True)
            bits = m.forward_masks(xd, packed=True)
        masks = masks.cpu().numpy().astype(bool)
        unpacked = np.unpackbits(bits.cpu().numpy(), axis=-1, bitorder="little").astype(bool)
        assert np.array_equal(unpacked, masks), "bit-packed and u8 masks disagree"
        ious = [orc.mask_iou(masks[i, k], ref_masks[i, k]) for i in range(2) for k in range(3)]
        print(f"512x512 {dtype}: logits rel err {rel_err(logits.cpu().numpy(), ref_logits):.3e}, "
              f"mask IoU min {min(ious):.5f} mean {np.mean(ious):.5f}")
        assert min(ious) >= min_iou
        m.close()


def test_masks_512_pretrained_weights():
    """Trained-like weights (synthetic profile "pretrained": bimodal logits, as a trained net
    has): fused masks of every dtype vs the fp32 CPU oracle at 512x512 (north_star IoU
    target 0.999)."""
    x = syn.invoice_pages(1000, 2, 512, 512, 3)
    sd = syn.make_state_dict(0, 3, 3, profile="pretrained")
    ref_logits = orc.unet_forward(sd, torch.from_numpy(x)).numpy()
    ref_masks = np.stack([np.stack(list(orc.masks_from_logits(ref_logits[i]).values())) for i in range(2)])
    assert 0.02 < ref_masks.mean() < 0.5
    xd = torch.from_numpy(x).to(DEV)
    for dtype, min_iou in (("fp32", 0.9999), ("fp16", 0.999), ("bf16", 0.99)):
        m = make_model(sd, 3, dtype)
        with torch.no_grad():
            bits = m.forward_masks(xd, packed=True)
        masks = np.unpackbits(bits.cpu().numpy(), axis=-1, bitorder="little").astype(bool)
        ious = [orc.mask_iou(masks[i, k], ref_masks[i, k]) for i in range(2) for k in range(3)]
        print(f"512x512 pretrained {dtype}: mask IoU min {min(ious):.5f} mean {np.mean(ious):.5f}")
        assert min(ious) >= min_iou
        m.close()


def test_run_unet_boundary_matches_reference_golden():
    """inference.run_unet (drop-in) on the golden 600x400 photo vs the reference's masks/crops."""
    from PIL import Image
    import hashlib
    from unet_mi355x import inference as inf
    z = np.load(os.path.join(GOLD, "run_unet_600x400.npz"))
    sd = syn.make_state_dict(int(z["seed"]), 3, 3, profile="structured")
    sd["out_conv.bias"] = sd["out_conv.bias"] + z["out_bias_delta"]
    assert syn.state_dict_checksum(sd) == str(z["sd_sha256"])
    pil = Image.fromarray(z["image"], mode="RGB")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, ck)
        inf.DEVICE = DEV
        masks, crops = inf.run_unet(pil, ck, compute_dtype="fp32")
    for k in inf.FIELDS:
        ref = np.unpackbits(z["maskbits_" + k], axis=-1, bitorder="little").astype(bool)
        iou = orc.mask_iou(masks[k], ref)
        print(f"run_unet {k}: IoU {iou:.6f}, differing pixels {int((masks[k] != ref).sum())}")
        assert iou >= 0.999
        if bool(z["crop_none_" + k]):
            assert crops[k] is None
        else:
            arr = np.asarray(crops[k])
            assert list(arr.shape) == list(z["crop_shape_" + k])
            if np.array_equal(masks[k], ref):
                assert hashlib.sha256(arr.tobytes()).hexdigest() == str(z["crop_sha256_" + k])


def test_errors_and_no_fallback():
    m = make_model(syn.make_state_dict(0, 3, 3), 3, "bf16")
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 40, 32, device=DEV))
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 32, 32))
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 1, 32, 32, device=DEV))
    m.close()


def test_weight_update_repacks():
    sd = syn.make_state_dict(4, 3, 3)
    m = make_model(sd, 3, "fp32")
    x = torch.from_numpy(syn.uniform_batch(1, 1, 3, 32, 32)).to(DEV)
    with torch.no_grad():
        a = m(x).clone()
        m.out_conv.bias.add_(1.0)
        b = m(x)
    assert torch.allclose(b - a, torch.ones_like(a), atol=1e-4)
    m.close()


@pytest.mark.parametrize("cfg", list(range(34)))
def test_every_kernel_config(cfg, monkeypatch):
    """Each implicit-GEMM configuration (csrc/unet_internal.h Cfg) forced on every 3x3 layer
    it supports, checked against the reference golden (fp32 and bf16)."""
    monkeypatch.setenv("UNET_MI355X_CFG", ",".join(f"{i}:{cfg}" for i in range(17)))
    z = np.load(os.path.join(GOLD, "unet_c3_h64w64_n2_structured.npz"))
    sd = syn.make_state_dict(int(z["seed"]), 3, 3, profile=str(z["profile"]))
    for dtype in ("fp32", "bf16"):
        m = make_model(sd, 3, dtype)
        with torch.no_grad():
            out = m(torch.from_numpy(z["x"]).to(DEV)).cpu().numpy()
        err = rel_err(out, z["logits"])
        print(f"cfg {cfg} {dtype}: rel err {err:.3e}")
        assert err <= TOL[dtype]
        m.close()


@pytest.mark.parametrize("cfg", [0, 1, 4, 5, 8, 9, 14, 15, 21, 22, 32, 34, 35, 36])
def test_convtranspose_configs(cfg, monkeypatch):
    """ConvTranspose2d (up4..up1) on every supported kernel configuration vs the golden."""
    monkeypatch.setenv("UNET_MI355X_UPCFG", ",".join(f"{i}:{cfg}" for i in range(4)))
    z = np.load(os.path.join(GOLD, "unet_c3_h16w16_n3_structured.npz"))
    sd = syn.make_state_dict(int(z["seed"]), 3, 3, profile=str(z["profile"]))
    for dtype in ("fp32", "bf16"):
        m = make_model(sd, 3, dtype)
        with torch.no_grad():
            out = m(torch.from_numpy(z["x"]).to(DEV)).cpu().numpy()
        for name, key in (("u1", "inter_u1_up"), ("u4", "inter_u4_up")):
            ref = z[key]
            got = m.intermediate(name).cpu().numpy().reshape(ref.shape)
            assert rel_err(got, ref) <= TOL[dtype], (cfg, dtype, name)
        assert rel_err(out, z["logits"]) <= TOL[dtype]
        m.close()


INTER = ["c1", "p1", "c2", "p2", "c3", "p3", "c4", "p4", "bn", "u4", "u3", "u2", "c7", "u1", "c8a"]


def _forward_state(m, x):
    with torch.no_grad():
        lg = m(x)
    torch.cuda.synchronize()
    out = {k: m.intermediate(k).clone() for k in INTER}
    out["logits"] = lg.clone()
    return out


def _first_diff(a, b):
    return [k for k in INTER + ["logits"] if not torch.equal(a[k], b[k])]


def _forced(cfg, up, sd, x, dtype, monkeypatch):
    monkeypatch.setenv("UNET_MI355X_CFG", ",".join(f"{i}:{cfg}" for i in range(17)) if cfg is not None else "")
    monkeypatch.setenv("UNET_MI355X_UPCFG", ",".join(f"{i}:{up}" for i in range(4)) if up is not None else "")
    m = make_model(sd, 3, dtype)
    st = _forward_state(m, x)
    m.close()
    return st


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_forward_deterministic_and_config_invariant(dtype, monkeypatch):
    """Full-size pages (persistent kernels walk several tiles per block, rings wrap): repeated
    forwards are bitwise identical, and within each kernel family every configuration --
    forced on all 3x3 layers, or on all ConvTranspose layers -- gives bitwise the same
    activations: the 128-byte LDS-halo configurations 4..26 (K order chunk64-major /
    tap-minor) agree with each other, the 64-byte ring configurations 27..31 and 33 (chunk32-major; 33 = down1.0 fused)
    agree with each other, and the ConvTranspose configurations agree with the defaults.  A
    missed wait in a DMA ring shows up here as a run-to-run or config-to-config difference."""
    x = torch.from_numpy(syn.invoice_pages(3, 2, 512, 512, 3)).to(DEV)
    sd = syn.make_state_dict(3, 3, 3, profile="structured")
    m = make_model(sd, 3, dtype)
    base = _forward_state(m, x)
    for r in range(2):
        assert _first_diff(_forward_state(m, x), base) == [], f"run {r + 1} differs"
    m.close()
    bad = []
    for family in (list(range(4, 27)), list(range(27, 32)) + [33]):
        fbase = _forced(family[0], None, sd, x, dtype, monkeypatch)
        for cfg in family[1:]:
            d = _first_diff(_forced(cfg, None, sd, x, dtype, monkeypatch), fbase)
            if d:
                bad.append((cfg, None, d[:3]))
    for up in (4, 5, 8, 9, 14, 15, 21, 22, 23, 25, 32, 34, 35, 36):
        d = _first_diff(_forced(None, up, sd, x, dtype, monkeypatch), base)
        if d:
            bad.append((None, up, d[:3]))
    print(bad)
    assert bad == []


def _np_boxes(masks):
    """[N, C, H, W] bool -> int32 [N, C, 4] (x_min, y_min, x_max, y_max), -1s if empty."""
    out = np.full(masks.shape[:2] + (4,), -1, dtype=np.int32)
    for i in range(masks.shape[0]):
        for c in range(masks.shape[1]):
            ys, xs = np.where(masks[i, c])
            if len(xs):
                out[i, c] = (xs.min(), ys.min(), xs.max(), ys.max())
    return out


@pytest.mark.parametrize("kind", [None, "u8", "bits"])
def test_mask_boxes_match_numpy(kind):
    """Device per-(image, field) boxes (unet_forward_boxes) == np.where min/max of the masks the
    same forward produced (inference.py:84-90), with and without caller mask buffers; empty
    masks (torch_default weights: logits ~ -4) give -1s; W = 48 exercises a 16-bit word row."""
    cases = [(syn.make_state_dict(0, 3, 3, "pretrained"), syn.invoice_pages(1000, 2, 512, 512, 3)),
             (syn.make_state_dict(1, 3, 3, "torch_default"), syn.invoice_pages(2, 1, 64, 64, 3)),
             (syn.make_state_dict(5, 3, 3, "structured", out_bias=0.0), syn.uniform_batch(3, 3, 3, 32, 48))]
    for sd, x in cases:
        m = make_model(sd, 3, "bf16")
        xd = torch.from_numpy(x).to(DEV)
        with torch.no_grad():
            ref_masks = m.forward_masks(xd).cpu().numpy().astype(bool)
            got = m.forward_boxes(xd, masks=kind)
        boxes = (got if kind is None else got[1]).cpu().numpy()
        assert np.array_equal(boxes, _np_boxes(ref_masks))
        if kind is not None:
            mk = got[0].cpu().numpy()
            if kind == "bits":
                mk = np.unpackbits(mk, axis=-1, bitorder="little")
            assert np.array_equal(mk.astype(bool), ref_masks)
        m.close()


def test_config5_1024_fp16():
    """BASELINE config 5 shape (1024x1024, 3 channels, 5 resolution levels, fp16 storage with
    fp32 accumulation): logits vs the fp32 CPU oracle and fused masks (IoU) on one page; a
    batch of 3 agrees with the single-image forward bitwise (no cross-image coupling)."""
    x = syn.invoice_pages(1000, 1, 1024, 1024, 3)
    sd = syn.make_state_dict(0, 3, 3, profile="pretrained")
    ref = orc.unet_forward(sd, torch.from_numpy(x)).numpy()
    ref_masks = np.stack(list(orc.masks_from_logits(ref[0]).values()))
    m = make_model(sd, 3, "fp16")
    xd = torch.from_numpy(x).to(DEV)
    with torch.no_grad():
        masks, logits = m.forward_masks(xd, with_logits=True)
        x3 = torch.cat([torch.from_numpy(syn.invoice_pages(7, 1, 1024, 1024, 3)).to(DEV), xd,
                        torch.from_numpy(syn.uniform_batch(2, 1, 3, 1024, 1024)).to(DEV)])
        lg3 = m(x3)
    err = rel_err(logits.cpu().numpy(), ref)
    ious = [orc.mask_iou(masks[0, k].cpu().numpy().astype(bool), ref_masks[k]) for k in range(3)]
    print(f"1024x1024 fp16: logits rel err {err:.3e}, mask IoU {ious}")
    assert err <= TOL["fp16"]
    assert min(ious) >= 0.995
    assert torch.equal(lg3[1:2], logits)
    m.close()


@pytest.mark.parametrize("h,w,c", [(400, 600, 3), (1333, 1000, 3), (200, 300, 3), (700, 512, 3),
                                   (512, 900, 3), (512, 512, 3), (390, 517, 1), (37, 23, 3), (3024, 4032, 3)])
def test_preprocess_bit_exact_with_pillow(h, w, c):
    """unet_preprocess (GPU) == PIL Image.resize((512, 512)) (default BICUBIC) + convert("RGB")
    + /255, bit for bit: down / up / one-axis / identity geometries, RGB and L, a 12 MP photo."""
    from PIL import Image
    rng = np.random.default_rng(h + 3 * w)
    arr = rng.integers(0, 256, (h, w, c) if c == 3 else (h, w), dtype=np.uint8)
    if h == 3024:   # smooth photo-like content (strong low-pass response, clip8 at both ends)
        yy, xx = np.mgrid[0:h, 0:w]
        arr = (127.5 + 127.5 * (np.sin(yy / 37.0) * np.cos(xx / 53.0))[..., None] + rng.normal(0, 20, (h, w, 3))
               ).clip(0, 255).astype(np.uint8)
    pil = Image.fromarray(arr)
    ref = np.array(pil.resize((512, 512)).convert("RGB")).astype(np.float32) / 255.0
    m = make_model(syn.make_state_dict(0, 3, 3), 3, "bf16")
    got = m.preprocess(torch.from_numpy(arr).to(DEV)).cpu().numpy()[0]
    assert got.shape == (3, 512, 512)
    assert np.array_equal(got, ref.transpose(2, 0, 1))
    if h < 2000:   # the numpy restatement agrees too (checker of the checker)
        from oracle import pil_resample as pr
        assert np.array_equal(got, pr.to_input(arr))
    m.close()


def test_run_unet_batch_equals_per_photo_calls():
    """inference.run_unet_batch (one forward over N photos of mixed sizes / modes) returns, for
    every photo, exactly run_unet's masks and crops."""
    from PIL import Image
    from unet_mi355x import inference as inf
    rng = np.random.default_rng(9)
    pages = syn.invoice_pages(1000, 3, 512, 512, 1)
    photos = [Image.fromarray((pages[0, 0] * 255).astype(np.uint8)).resize((600, 400)).convert("RGB"),
              Image.fromarray((pages[1, 0] * 255).astype(np.uint8)).resize((300, 700)),            # mode L
              Image.fromarray(rng.integers(0, 256, (333, 517, 4), dtype=np.uint8), mode="RGBA")]  # host path
    sd = syn.make_state_dict(0, 3, 3, "pretrained")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, ck)
        inf.DEVICE = DEV
        single = [inf.run_unet(p, ck, compute_dtype="bf16") for p in photos]
        batch = inf.run_unet_batch(photos, ck, compute_dtype="bf16")
    assert len(batch) == len(photos)
    for (m1, c1), (m2, c2) in zip(single, batch):
        for k in inf.FIELDS:
            assert np.array_equal(m1[k], m2[k]), k
            assert (c1[k] is None) == (c2[k] is None), k
            if c1[k] is not None:
                assert np.array_equal(np.asarray(c1[k]), np.asarray(c2[k])), k
