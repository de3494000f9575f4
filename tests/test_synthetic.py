"""Portable synthetic data generator (weights + invoice pages)."""
import numpy as np

from unet_mi355x import synthetic as syn


def test_key_set_matches_reference_layout():
    keys = [k for k, _ in syn.unet_shapes(3, 3)]
    assert len(keys) == 136 and len(set(keys)) == 136
    assert keys[0] == "down1.net.0.weight" and keys[-1] == "out_conv.bias"
    shapes = dict(syn.unet_shapes(3, 3))
    assert shapes["conv4.net.0.weight"] == (512, 1024, 3, 3)   # in_channels 1024 = cat(up4, c4)
    assert shapes["up4.weight"] == (1024, 512, 2, 2)           # ConvTranspose2d (Cin, Cout, 2, 2)


def test_deterministic_and_seed_sensitive():
    a = syn.uniform(1, "k", 1000)
    assert np.array_equal(a, syn.uniform(1, "k", 1000))
    assert not np.array_equal(a, syn.uniform(2, "k", 1000))
    assert 0.0 <= a.min() and a.max() < 1.0
    n = syn.normal(5, "z", 200000)
    assert abs(n.mean()) < 0.01 and abs(n.std() - 1) < 0.01
    # counter-based: a window equals the slice of a longer stream
    assert np.array_equal(syn.uniform(3, "w", 10, offset=5), syn.uniform(3, "w", 15)[5:])


def test_invoice_pages_range_and_gray_replication():
    p = syn.invoice_pages(0, 2, 64, 96, 3)
    assert p.shape == (2, 3, 64, 96) and p.dtype == np.float32
    assert p.min() >= 0 and p.max() <= 1
    assert np.array_equal(p[:, 0], p[:, 1]) and np.array_equal(p[:, 0], p[:, 2])
    assert (p < 0.35).mean() > 0.002   # dark "text" rectangles exist
