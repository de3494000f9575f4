"""The Pillow BICUBIC resize restatement (oracle/pil_resample.py) is bit-exact with the installed
Pillow -- the reference's own resize (inference.py:35,63) -- on up/down/one-axis/identity
geometries and RGB / L images.  It is the checker of the device resampler (-m gpu tests)."""
import numpy as np
import pytest
from PIL import Image

from oracle import pil_resample as pr


@pytest.mark.parametrize("h,w,c", [(400, 600, 3), (1333, 1000, 3), (200, 300, 3), (700, 512, 3),
                                   (512, 900, 3), (512, 512, 3), (390, 517, 1), (37, 23, 3)])
def test_restatement_matches_pillow(h, w, c):
    rng = np.random.default_rng(h * 7 + w)
    arr = rng.integers(0, 256, (h, w, c) if c == 3 else (h, w), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(arr).resize((512, 512)))
    assert np.array_equal(pr.resize(arr, 512, 512), ref)


def test_to_input_matches_reference_preprocess_arithmetic():
    rng = np.random.default_rng(3)
    arr = rng.integers(0, 256, (300, 200), dtype=np.uint8)
    img = Image.fromarray(arr).resize((512, 512))          # inference.py:63 (mode L)
    ref = np.array(img.convert("RGB").resize((512, 512))).astype(np.float32) / 255.0   # :35-36
    assert np.array_equal(pr.to_input(arr), ref.transpose(2, 0, 1))
