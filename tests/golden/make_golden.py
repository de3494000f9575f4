"""Generate the golden fixtures by running the REFERENCE itself (survey container only).

Usage (from the repo root, where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only-pretrained]

It imports ``unet_model`` and ``inference`` from /root/reference (SURVEY.md §8c:
importable, nothing denied), loads seeded synthetic weights (the real
checkpoint is an LFS pointer) into the reference ``UNet`` with a strict
``load_state_dict``, and stores inputs + reference outputs as small ``.npz``
data files.  No reference source is copied; only its outputs are kept.
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
from unet_mi355x import synthetic as syn  # noqa: E402

REF = "/root/reference"


def ref_modules():
    sys.path.insert(0, REF)
    import unet_model as ref_unet  # noqa: E402
    import inference as ref_inf    # noqa: E402
    sys.path.remove(REF)
    return ref_unet, ref_inf


def to_torch_sd(sd):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}


def build(ref_unet, sd, n_channels, n_classes):
    m = ref_unet.UNet(n_channels=n_channels, n_classes=n_classes)
    m.load_state_dict(to_torch_sd(sd), strict=True)
    return m.eval()


def forward_with_hooks(model, x):
    inter = {}
    names = {"down1": "c1", "down2": "c2", "down3": "c3", "down4": "c4", "bottleneck": "bn",
             "conv4": "c5", "conv3": "c6", "conv2": "c7", "conv1": "c8", "up1": "u1_up", "up4": "u4_up"}
    hs = [getattr(model, mod).register_forward_hook(
        lambda m, i, o, key=key: inter.__setitem__(key, o.detach().clone()))
        for mod, key in names.items()]
    with torch.no_grad():
        out = model(x)
    for h in hs:
        h.remove()
    return out, inter


PRETRAINED_512_PAGES = (0, 13, 37, 63)    # indices into the bench's 64 unique pages (bench.gen_pages seed 1000)


def quantised_pages(seed, n, size):
    """Invoice pages as a photo would deliver them: uint8 gray (x255, round half up), replicated
    x3.  x = u8 / 255 is then exactly what inference.preprocess produces for that photo."""
    pages = syn.invoice_pages(seed, n, size, size, 1)[:, 0]
    return (pages.astype(np.float64) * 255.0 + 0.5).astype(np.uint8)


def pretrained_cases(ref_unet, ref_inf):
    """The benchmarked shapes pinned to the reference: the trained-like
    "pretrained" weight profile the bench's IoU claims use, on the bench's own pages.

    * pretrained_512_pages.npz: 4 of the bench's 512x512 pages (uint8-quantised), masks from the
      REFERENCE's run_unet (inference.py:50-79: load_model, resize, preprocess, forward, sigmoid,
      per-field thresholds) as bit-packed arrays, its 1/8-subsampled logits, and the sha256 of
      the network input preprocess() built.
    * pretrained_1024_page.npz: one 1024x1024 page (BASELINE config 5 shape) through the
      reference UNet.forward; masks with inference.py:72-79's sigmoid + thresholds applied to it.
    """
    import hashlib
    from PIL import Image
    sd = syn.make_state_dict(0, 3, 3, profile="pretrained")
    u8 = quantised_pages(1000, max(PRETRAINED_512_PAGES) + 1, 512)[list(PRETRAINED_512_PAGES)]
    model = build(ref_unet, sd, 3, 3)
    payload = dict(page_index=np.array(PRETRAINED_512_PAGES, np.int64), pages_u8=u8,
                   sd_sha256=np.array(syn.state_dict_checksum(sd)), profile=np.array("pretrained"))
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "ckpt.pth")
        torch.save(to_torch_sd(sd), ck)
        ref_inf.DEVICE = "cpu"
        for j, page in enumerate(u8):
            pil = Image.fromarray(np.stack([page] * 3, axis=-1), mode="RGB")
            masks, _ = ref_inf.run_unet(pil, ck)
            x = ref_inf.preprocess(pil.resize((512, 512)))
            assert np.array_equal(x.numpy()[0, 0], page.astype(np.float32) / 255.0)
            with torch.no_grad():
                logits = model(x)[0].numpy()
            payload[f"x_sha256_{j}"] = np.array(hashlib.sha256(x.numpy().tobytes()).hexdigest())
            payload[f"logits_sub8_{j}"] = logits[:, ::8, ::8].copy()
            for k in ref_inf.FIELDS:
                payload[f"maskbits_{k}_{j}"] = np.packbits(masks[k].astype(np.uint8), axis=-1, bitorder="little")
            print("pretrained_512 page", PRETRAINED_512_PAGES[j], {k: round(float(masks[k].mean()), 4) for k in masks})
    np.savez_compressed(os.path.join(HERE, "pretrained_512_pages.npz"), **payload)

    page = quantised_pages(1000, 1, 1024)[0]
    x = torch.from_numpy(np.ascontiguousarray(np.stack([page] * 3)[None].astype(np.float32) / 255.0))
    with torch.no_grad():
        logits = model(x)
        prob = torch.sigmoid(logits.squeeze(0)).numpy()
    thr = {"invoice_no": 0.25, "date": 0.40, "total_amount": 0.30}    # inference.py:76-78
    payload = dict(page_u8=page, sd_sha256=np.array(syn.state_dict_checksum(sd)), profile=np.array("pretrained"),
                   logits_sub8=logits[0].numpy()[:, ::8, ::8].copy())
    for i, k in enumerate(ref_inf.FIELDS):
        payload[f"maskbits_{k}"] = np.packbits((prob[i] > thr[k]).astype(np.uint8), axis=-1, bitorder="little")
    np.savez_compressed(os.path.join(HERE, "pretrained_1024_page.npz"), **payload)
    print("pretrained_1024", {k: round(float((prob[i] > thr[k]).mean()), 4) for i, k in enumerate(ref_inf.FIELDS)})


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref_unet, ref_inf = ref_modules()
    if "--only-pretrained" in sys.argv:
        pretrained_cases(ref_unet, ref_inf)
        return
    cases = [
        # name, n_channels, H, W, N, profile, seed, input kind, keep intermediates
        ("unet_c3_h64w64_n2_structured", 3, 64, 64, 2, "structured", 1, "invoice", False),
        ("unet_c1_h32w48_n2_structured", 1, 32, 48, 2, "structured", 2, "uniform", False),
        ("unet_c3_h48w32_n1_default", 3, 48, 32, 1, "torch_default", 3, "uniform", False),
        ("unet_c3_h16w16_n3_structured", 3, 16, 16, 3, "structured", 4, "uniform", True),
    ]
    for name, c, h, w, n, prof, seed, kind, keep in cases:
        sd = syn.make_state_dict(seed, c, 3, profile=prof)
        x = syn.invoice_pages(seed, n, h, w, c) if kind == "invoice" else syn.uniform_batch(seed, n, c, h, w)
        model = build(ref_unet, sd, c, 3)
        out, inter = forward_with_hooks(model, torch.from_numpy(x))
        payload = dict(x=x, logits=out.numpy(), seed=np.int64(seed), n_channels=np.int64(c),
                       profile=np.array(prof), sd_sha256=np.array(syn.state_dict_checksum(sd)))
        if keep:
            for k, v in inter.items():
                payload["inter_" + k] = v.numpy()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **payload)
        print(name, {k: getattr(v, "shape", None) for k, v in payload.items()})

    # Full-size 512x512 forward + the run_unet boundary (inference.py:50-129) on a
    # seeded 600x400 photo.  out_conv bias is re-centred so that masks are non-empty.
    from PIL import Image
    seed = 7
    page = syn.invoice_pages(seed, 1, 400, 600, 1)[0, 0]
    rgb = np.stack([page, page * 0.97, page * 0.94], axis=-1)
    pil = Image.fromarray((rgb * 255.0 + 0.5).astype(np.uint8), mode="RGB")
    sd = syn.make_state_dict(seed, 3, 3, profile="structured")
    model = build(ref_unet, sd, 3, 3)
    x = ref_inf.preprocess(pil.resize((512, 512)))
    with torch.no_grad():
        logits = model(x)[0].numpy()
    # bias so that roughly 10% of each channel is above its threshold
    thr = np.array([0.25, 0.40, 0.30], dtype=np.float64)
    thr_logit = np.log(thr / (1 - thr))
    q = np.quantile(logits.reshape(3, -1).astype(np.float64), 0.90, axis=1)
    bias = (thr_logit - q).astype(np.float32)
    sd["out_conv.bias"] = sd["out_conv.bias"] + bias
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "ckpt.pth")
        torch.save(to_torch_sd(sd), ck)
        ref_inf.DEVICE = "cpu"
        masks, crops = ref_inf.run_unet(pil, ck)
        model = ref_inf.load_model(ck)
        with torch.no_grad():
            logits = model(x)[0].numpy()
    import hashlib
    payload = dict(image=np.asarray(pil), x_sub8=x.numpy()[0, :, ::8, ::8].copy(),
                   x_sha256=np.array(hashlib.sha256(x.numpy().tobytes()).hexdigest()),
                   out_bias_delta=bias, seed=np.int64(seed),
                   sd_sha256=np.array(syn.state_dict_checksum(sd)),
                   logits_sub4=logits[:, ::4, ::4].copy(),
                   logits_row0=logits[:, 0, :].copy(), logits_row257=logits[:, 257, :].copy())
    for i, k in enumerate(["invoice_no", "date", "total_amount"]):
        payload["maskbits_" + k] = np.packbits(masks[k].astype(np.uint8), axis=-1, bitorder="little")
        cr = crops[k]
        arr = np.zeros((0, 0, 3), np.uint8) if cr is None else np.asarray(cr)
        payload["crop_shape_" + k] = np.array(arr.shape, np.int64)
        payload["crop_sha256_" + k] = np.array(hashlib.sha256(arr.tobytes()).hexdigest())
        payload["crop_none_" + k] = np.bool_(cr is None)
    np.savez_compressed(os.path.join(HERE, "run_unet_600x400.npz"), **payload)
    print("run_unet_600x400", {k: (masks[k].mean(), None if crops[k] is None else crops[k].size) for k in masks})
    pretrained_cases(ref_unet, ref_inf)


if __name__ == "__main__":
    main()
