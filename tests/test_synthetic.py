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


def test_invoice_fields_follow_page_rectangles():
    p = syn.invoice_pages(4, 2, 128, 128, 1)
    f = syn.invoice_fields(4, 2, 128, 128)
    assert f.shape == (2, 3, 128, 128) and f.dtype == np.uint8
    on = f.max(axis=1).astype(bool)
    # every field pixel lies on a dark rectangle (noise is N(0, 0.02) around values <= 0.3)
    assert on.any() and (p[:, 0][on] < 0.45).all()
    assert f[:, 2].sum() > 0 and f[:, 0].sum() > 0


def test_pretrained_profile_is_the_structured_base_plus_the_committed_delta():
    base = syn.make_state_dict(0, 3, 3, "structured")
    pre = syn.make_state_dict(0, 3, 3, "pretrained")
    assert list(pre) == list(base)
    changed = [k for k in base if not np.array_equal(base[k], pre[k])]
    assert changed and all((".net.1." in k or ".net.4." in k or k.startswith("up") or k.startswith("out_conv"))
                           for k in changed)
    assert all(not k.endswith("running_mean") and not k.endswith("running_var") for k in changed)
    assert sum(pre[k].size for k in changed) < 20000
    # 3x3 conv and ConvTranspose weights stay the seeded ones
    assert np.array_equal(pre["conv4.net.0.weight"], base["conv4.net.0.weight"])
    assert np.array_equal(pre["up1.weight"], base["up1.weight"])
    one = syn.make_state_dict(0, 1, 3, "pretrained")
    assert one["down1.net.0.weight"].shape == (64, 1, 3, 3)
    assert np.array_equal(one["conv1.net.4.weight"], pre["conv1.net.4.weight"])
