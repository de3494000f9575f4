"""Give the synthetic UNet weights a trained-like logit distribution (data generator, not product).

The reference's trained checkpoint is a Git-LFS pointer, and the seeded
"structured" weights are untrained: their logits are unimodal around the thresholds, so
~20 % of pixels sit within rounding distance of a mask cut and any 16-bit forward path
shows an IoU against the fp32 CPU reference far below what a trained net would give
(hard part 1).  This tool fine-tunes a SMALL parameter subset of the
seed-0 structured weights -- every BatchNorm affine (gamma, beta), the ConvTranspose
biases and the 1x1 out_conv (~13 k of 31 M parameters, "BitFit") -- on the synthetic
invoice fields of ``synthetic.invoice_fields``, with the 3x3 / ConvTranspose weights
frozen at their seeded values.  The result is a committed 60 KB delta
(``unet_mi355x/data/pretrained_delta.npz``) that ``synthetic.make_state_dict(profile=
"pretrained")`` applies on top of the seed-0 weights.

Training runs on this container's CPU, fp32, eval-mode BN (the running stats stay the
seeded ones).  The model here is a plain torch.nn.functional restatement of
``unet_model.py:55-86`` (kept separate from oracle/, which is test infrastructure).

    python tools/pretrain_synthetic.py [--steps 300] [--crop 128] [--batch 8]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from unet_mi355x import synthetic as syn  # noqa: E402

BLOCKS = ("down1", "down2", "down3", "down4", "bottleneck", "conv4", "conv3", "conv2", "conv1")


def trainable(key: str) -> bool:
    return (".net.1." in key or ".net.4." in key) and key.rsplit(".", 1)[1] in ("weight", "bias") \
        or (key.startswith("up") and key.endswith(".bias")) or key.startswith("out_conv.")


def forward(p, x):
    def dc(name, t):
        for i in (0, 3):
            t = F.conv2d(t, p[f"{name}.net.{i}.weight"], p[f"{name}.net.{i}.bias"], padding=1)
            b = f"{name}.net.{i + 1}"
            t = F.batch_norm(t, p[f"{b}.running_mean"], p[f"{b}.running_var"], p[f"{b}.weight"],
                             p[f"{b}.bias"], training=False, eps=1e-5)
            t = F.relu(t)
        return t

    def up(name, t):
        return F.conv_transpose2d(t, p[f"{name}.weight"], p[f"{name}.bias"], stride=2)

    c1 = dc("down1", x)
    c2 = dc("down2", F.max_pool2d(c1, 2))
    c3 = dc("down3", F.max_pool2d(c2, 2))
    c4 = dc("down4", F.max_pool2d(c3, 2))
    bn = dc("bottleneck", F.max_pool2d(c4, 2))
    c7 = dc("conv4", torch.cat([up("up4", bn), c4], 1))
    c8 = dc("conv3", torch.cat([up("up3", c7), c3], 1))
    c9 = dc("conv2", torch.cat([up("up2", c8), c2], 1))
    c10 = dc("conv1", torch.cat([up("up1", c9), c1], 1))
    return F.conv2d(c10, p["out_conv.weight"], p["out_conv.bias"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--crop", type=int, default=128)
    ap.add_argument("--pages", type=int, default=48)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--out", default=os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd", "unet_mi355x", "data",
                                                  "pretrained_delta.npz"))
    a = ap.parse_args()
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count() or 1)
    sd = syn.make_state_dict(0, 3, 3, "structured")
    p = {k: torch.from_numpy(np.asarray(v, dtype=np.float32).copy()) for k, v in sd.items()
         if not k.endswith("num_batches_tracked")}
    train_keys = [k for k in p if trainable(k)]
    for k in train_keys:
        p[k].requires_grad_(True)
    print(f"trainable: {len(train_keys)} tensors, {sum(p[k].numel() for k in train_keys)} parameters", flush=True)

    pages = torch.from_numpy(syn.invoice_pages(7, a.pages, 512, 512, 3))
    fields = torch.from_numpy(syn.invoice_fields(7, a.pages, 512, 512)).float()
    pos = fields.mean(dim=(0, 2, 3))
    pos_weight = ((1 - pos) / pos.clamp_min(1e-3)).clamp(max=10.0).view(1, 3, 1, 1)
    print("field positive fractions", pos.tolist(), flush=True)
    rng = np.random.default_rng(0)
    opt = torch.optim.Adam([p[k] for k in train_keys], lr=a.lr)
    t0 = time.time()
    for step in range(a.steps):
        idx = rng.integers(0, a.pages, a.batch)
        ys = rng.integers(0, 512 - a.crop + 1, a.batch)
        xs = rng.integers(0, 512 - a.crop + 1, a.batch)
        xb = torch.stack([pages[i, :, y:y + a.crop, x:x + a.crop] for i, y, x in zip(idx, ys, xs)])
        yb = torch.stack([fields[i, :, y:y + a.crop, x:x + a.crop] for i, y, x in zip(idx, ys, xs)])
        logits = forward(p, xb)
        loss = F.binary_cross_entropy_with_logits(logits, yb, pos_weight=pos_weight)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if step % 20 == 0 or step == a.steps - 1:
            with torch.no_grad():
                acc = ((logits > 0) == (yb > 0.5)).float().mean().item()
                lo = logits.detach().flatten()
            print(f"step {step:4d} loss {loss.item():.4f} pixel-acc {acc:.4f} logit q01/q50/q99 "
                  f"{lo.quantile(0.01).item():.2f}/{lo.quantile(0.5).item():.2f}/{lo.quantile(0.99).item():.2f} "
                  f"({time.time() - t0:.0f}s)", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez_compressed(a.out, **{k: p[k].detach().numpy().astype(np.float32) for k in train_keys},
                        __base_checksum__=np.frombuffer(syn.state_dict_checksum(sd).encode(), dtype=np.uint8))
    print("wrote", a.out, os.path.getsize(a.out), "bytes")


if __name__ == "__main__":
    main()
