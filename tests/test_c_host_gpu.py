"""The boundary from a plain-C host (tests/c_host/unet_c_host.c): a process with no Python and no torch
creates a handle from include/unet_mi355x.h, loads the reference's 136-key state_dict from raw host
buffers, runs unet_forward_boxes eagerly and as a replayed graph (it checks those agree bit for bit),
and writes logits, masks and boxes -- which must equal the Python binding's forward of the same
weights bit for bit (same library, same plan)."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
from unet_mi355x import native, synthetic as syn  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402

BIN = os.path.join(REPO, "tests", "c_host", "unet_c_host")
DTYPES = {"fp32": native.DTYPES["fp32"], "mixed": native.DTYPES["mixed"]}


def write_inputs(d, sd, x, thresholds):
    """manifest.txt + weights.bin (the state_dict as raw host tensors) + x.bin, the C host's format."""
    lines = [" ".join([str(3)] + [repr(float(t)) for t in list(thresholds) + [0.5] * (4 - len(thresholds))])]
    off = 0
    with open(os.path.join(d, "weights.bin"), "wb") as f:
        for k, v in sd.items():
            a = np.ascontiguousarray(v)
            dt = 0 if a.dtype == np.float32 else 1
            shape = list(a.shape) + [0] * (4 - a.ndim)
            lines.append(f"{k} {dt} {a.ndim} {' '.join(str(s) for s in shape)} {off} {a.nbytes}")
            f.write(a.tobytes())
            off += a.nbytes
    with open(os.path.join(d, "manifest.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    np.ascontiguousarray(x, dtype=np.float32).tofile(os.path.join(d, "x.bin"))


@pytest.fixture(scope="module", autouse=True)
def c_host_binary():
    """Bring the C host up to date (`make c_host`: the library's own test target, incremental: it rebuilds
    only when the source, the header or the library changed); skip the module without a C compiler and
    no binary."""
    import shutil
    if shutil.which("make") is None or shutil.which(os.environ.get("CC", "cc")) is None:
        if not os.path.exists(BIN):
            pytest.skip("no C compiler to build tests/c_host/unet_c_host")
        return BIN
    r = subprocess.run(["make", "-C", os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd", "csrc"), "c_host"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return BIN


def test_c_host_binary_matches_the_header():
    """The C host links the library and agrees with the header's ABI version (no GPU call)."""
    r = subprocess.run([BIN, "--abi"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.split() == ["header", str(native.ABI_VERSION), "library", str(native.ABI_VERSION)]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["mixed", "fp32"])
def test_c_host_forward_equals_python_binding(dtype):
    sd = {k: np.asarray(v) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}
    n, hw = 2, 256
    x = syn.invoice_pages(41, n, hw, hw, 3)
    m = UNet(3, 3, compute_dtype=dtype)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to("cuda:0").eval()
    xd = torch.from_numpy(x).to("cuda:0")
    with torch.no_grad():
        logits = m(xd).cpu().numpy()
        masks, boxes = m.forward_boxes(xd, masks="u8")
    masks, boxes = masks.cpu().numpy(), boxes.cpu().numpy()
    m.close()
    with tempfile.TemporaryDirectory() as d:
        write_inputs(d, sd, x, m.thresholds)
        r = subprocess.run([BIN, d, str(DTYPES[dtype]), str(n), str(hw), str(hw)], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.startswith("ok: 136 tensors"), r.stdout
        c_logits = np.fromfile(os.path.join(d, "logits.bin"), np.float32).reshape(logits.shape)
        c_masks = np.fromfile(os.path.join(d, "masks.bin"), np.uint8).reshape(masks.shape)
        c_boxes = np.fromfile(os.path.join(d, "boxes.bin"), np.int32).reshape(boxes.shape)
    assert np.array_equal(c_logits, logits)
    assert np.array_equal(c_masks, masks)
    assert np.array_equal(c_boxes, boxes)
    assert (c_boxes[..., 2] >= 0).any()   # the pretrained-like weights find fields on the pages
