"""The oracle (CPU restatement, oracle/unet_oracle.py) against the golden vectors the
reference itself produced (tests/golden/make_golden.py).  CPU only."""
import glob
import hashlib
import os

import numpy as np
import pytest
import torch

from oracle import unet_oracle as orc
from unet_mi355x import synthetic as syn

GOLD = os.path.join(os.path.dirname(__file__), "golden")
UNET_CASES = sorted(glob.glob(os.path.join(GOLD, "unet_*.npz")))


def _sd_for(z):
    c = int(z["n_channels"])
    sd = syn.make_state_dict(int(z["seed"]), c, 3, profile=str(z["profile"]))
    assert syn.state_dict_checksum(sd) == str(z["sd_sha256"]), "synthetic weight generator drifted"
    return sd


@pytest.mark.parametrize("path", UNET_CASES, ids=os.path.basename)
def test_oracle_matches_reference_logits(path):
    z = np.load(path)
    sd = _sd_for(z)
    out, inter = orc.unet_forward(sd, torch.from_numpy(z["x"]), return_intermediates=True)
    ref = z["logits"]
    scale = max(1.0, float(np.abs(ref).max()))
    np.testing.assert_allclose(out.numpy(), ref, rtol=0, atol=2e-5 * scale)
    for k in z.files:
        if k.startswith("inter_") and k[6:] in inter:
            r = z[k]
            np.testing.assert_allclose(inter[k[6:]].numpy(), r, rtol=0, atol=2e-5 * max(1.0, float(np.abs(r).max())))


def test_oracle_rejects_non_multiple_of_16():
    sd = syn.make_state_dict(0, 3, 3)
    with pytest.raises(RuntimeError):
        orc.unet_forward(sd, torch.zeros(1, 3, 40, 32))


def test_run_unet_postprocess_matches_reference():
    """Oracle crop boxes + crops from the reference's own masks reproduce its crops."""
    z = np.load(os.path.join(GOLD, "run_unet_600x400.npz"))
    img = z["image"]
    oh, ow = img.shape[:2]
    masks = {k: np.unpackbits(z["maskbits_" + k], axis=-1, bitorder="little").astype(bool)
             for k in orc.FIELDS}
    boxes = orc.crop_boxes(masks, ow, oh)
    for k in orc.FIELDS:
        if bool(z["crop_none_" + k]):
            assert boxes[k] is None or img[boxes[k][1]:boxes[k][3], boxes[k][0]:boxes[k][2]].mean() < 3
            continue
        x1, y1, x2, y2 = boxes[k]
        crop = np.ascontiguousarray(img[y1:y2, x1:x2])
        assert list(crop.shape) == list(z["crop_shape_" + k])
        assert hashlib.sha256(crop.tobytes()).hexdigest() == str(z["crop_sha256_" + k])


def test_mask_threshold_semantics():
    """sigmoid + strict '>' in fp32 (inference.py:72-79)."""
    thr_logit = np.log(0.25 / 0.75)
    logits = np.zeros((3, 2, 2), np.float32)
    logits[0, 0, 0] = thr_logit + 1e-3
    logits[0, 0, 1] = thr_logit - 1e-3
    m = orc.masks_from_logits(logits)
    assert m["invoice_no"][0, 0] and not m["invoice_no"][0, 1]
    assert orc.mask_iou(m["date"], m["date"]) == 1.0


def test_oracle_matches_reference_512_logits():
    """Full-size parity of the oracle with the reference: the reference's own run_unet input for
    the golden 600x400 photo (PIL resize to 512 + inference.preprocess, pinned by its sha256) and
    its 512x512 logits (1/4-subsampled grid, rows 0 and 257; make_golden.py)."""
    from PIL import Image
    z = np.load(os.path.join(GOLD, "run_unet_600x400.npz"))
    sd = syn.make_state_dict(int(z["seed"]), 3, 3, profile="structured")
    sd["out_conv.bias"] = sd["out_conv.bias"] + z["out_bias_delta"]
    assert syn.state_dict_checksum(sd) == str(z["sd_sha256"])
    x = orc.preprocess(Image.fromarray(z["image"], mode="RGB").resize((512, 512)))
    assert hashlib.sha256(x.numpy().tobytes()).hexdigest() == str(z["x_sha256"])
    lg = orc.unet_forward(sd, x).numpy()[0]
    for got, key in ((lg[:, ::4, ::4], "logits_sub4"), (lg[:, 0, :], "logits_row0"), (lg[:, 257, :], "logits_row257")):
        ref = z[key]
        np.testing.assert_allclose(got, ref, rtol=0, atol=2e-5 * max(1.0, float(np.abs(ref).max())), err_msg=key)
    # and the masks / crops of the reference's run_unet follow from these logits
    masks = orc.masks_from_logits(lg)
    for k in orc.FIELDS:
        ref = np.unpackbits(z["maskbits_" + k], axis=-1, bitorder="little").astype(bool)
        assert orc.mask_iou(masks[k], ref) >= 0.9999, k


def test_oracle_run_unet_matches_reference_golden():
    """The CPU baseline's end-to-end leg (oracle.run_unet: checkpoint load, resize, forward,
    masks, crops -- inference.py:50-129) reproduces the reference's run_unet golden."""
    import tempfile
    from PIL import Image
    z = np.load(os.path.join(GOLD, "run_unet_600x400.npz"))
    sd = syn.make_state_dict(int(z["seed"]), 3, 3, profile="structured")
    sd["out_conv.bias"] = sd["out_conv.bias"] + z["out_bias_delta"]
    pil = Image.fromarray(z["image"], mode="RGB")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, ck)
        masks, crops = orc.run_unet(pil, ck)
    for k in orc.FIELDS:
        ref = np.unpackbits(z["maskbits_" + k], axis=-1, bitorder="little").astype(bool)
        assert orc.mask_iou(masks[k], ref) >= 0.9999, k
        if bool(z["crop_none_" + k]):
            assert crops[k] is None
        else:
            arr = np.asarray(crops[k])
            assert list(arr.shape) == list(z["crop_shape_" + k])
            if np.array_equal(masks[k], ref):
                assert hashlib.sha256(arr.tobytes()).hexdigest() == str(z["crop_sha256_" + k])


def _pretrained_sd(z):
    sd = syn.make_state_dict(0, 3, 3, profile="pretrained")
    assert syn.state_dict_checksum(sd) == str(z["sd_sha256"]), "pretrained weight profile drifted"
    return sd


def test_pretrained_pages_are_the_bench_pages():
    """The fixture pages are the bench's own pages (bench.gen_pages seed 1000, 64 unique pages),
    quantised to uint8 as a photo delivers them (make_golden.quantised_pages)."""
    import bench
    z = np.load(os.path.join(GOLD, "pretrained_512_pages.npz"))
    pages = bench.gen_pages(1000, 64, 512, 1, unique=64)[:, 0]
    for j, i in enumerate(z["page_index"]):
        q = (pages[i].astype(np.float64) * 255.0 + 0.5).astype(np.uint8)
        assert np.array_equal(q, z["pages_u8"][j])


def test_oracle_matches_reference_pretrained_512_pages():
    """The oracle on the trained-like weight profile the bench's IoU claims use, against the
    reference's own run_unet masks and logits for 4 of the bench's 512x512 pages."""
    z = np.load(os.path.join(GOLD, "pretrained_512_pages.npz"))
    sd = _pretrained_sd(z)
    x = torch.from_numpy(np.repeat(z["pages_u8"][:, None].astype(np.float32) / 255.0, 3, axis=1))
    lg = orc.unet_forward(sd, x).numpy()
    for j in range(x.shape[0]):
        assert hashlib.sha256(x[j:j + 1].numpy().tobytes()).hexdigest() == str(z[f"x_sha256_{j}"])
        ref = z[f"logits_sub8_{j}"]
        np.testing.assert_allclose(lg[j][:, ::8, ::8], ref, rtol=0, atol=2e-5 * max(1.0, float(np.abs(ref).max())))
        masks = orc.masks_from_logits(lg[j])
        for k in orc.FIELDS:
            refm = np.unpackbits(z[f"maskbits_{k}_{j}"], axis=-1, bitorder="little").astype(bool)
            assert orc.mask_iou(masks[k], refm) >= 0.9999, (j, k)


def test_oracle_matches_reference_pretrained_1024_page():
    """BASELINE config 5's resolution: one 1024x1024 page through the reference forward."""
    z = np.load(os.path.join(GOLD, "pretrained_1024_page.npz"))
    sd = _pretrained_sd(z)
    x = torch.from_numpy(np.repeat(z["page_u8"][None, None].astype(np.float32) / 255.0, 3, axis=1))
    lg = orc.unet_forward(sd, x).numpy()[0]
    ref = z["logits_sub8"]
    np.testing.assert_allclose(lg[:, ::8, ::8], ref, rtol=0, atol=2e-5 * max(1.0, float(np.abs(ref).max())))
    masks = orc.masks_from_logits(lg)
    for k in orc.FIELDS:
        refm = np.unpackbits(z[f"maskbits_{k}"], axis=-1, bitorder="little").astype(bool)
        assert orc.mask_iou(masks[k], refm) >= 0.9999, k
