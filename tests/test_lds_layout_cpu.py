"""The LDS bank model of down1.3's computed halo (tools/halo_swizzle_search.py) against the
kernel's layout: every halo pixel written exactly once, and the three accesses of the layer
(tap B-fragment reads, halo writes, first-conv window reads) at their modelled LDS cycles
(MI355X_MICROARCH.md §LDS bank rules).  CPU only: it checks the index arithmetic the kernel uses
(conv3x3_ring8_kernel, HS = 1, compute_halo / taps9), not the hardware."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import halo_swizzle_search as hs  # noqa: E402


def kernel_pixel(grp, c):
    """compute_halo's mapping, restated from unet_kernels.hip."""
    if grp < 36:
        rp = grp >> 2
        return 6 * (rp // 3) + rp % 3 + 3 * ((c >> 2) & 1), 8 * (grp & 3) + (c & 3) + 4 * (c >> 3)
    k = (grp - 36) * 16 + c
    return None if k >= 36 else (k >> 1, 32 + (k & 1))


def kernel_swizzle(hy, hx):
    return (hx & 3) ^ (hy & 1)


def test_kernel_halo_mapping_covers_every_pixel_once():
    seen = [kernel_pixel(g, c) for g in range(39) for c in range(16)]
    real = [p for p in seen if p is not None]
    assert len(real) == hs.HP == len(set(real))
    assert all(0 <= hy < 18 and 0 <= hx < hs.HWD for hy, hx in real)
    assert all(kernel_pixel(g, c) == hs.kernel_map(g, c) for g in range(39) for c in range(16))


def test_kernel_layout_is_conflict_free_where_round2_was_not():
    assert hs.tap_reads(kernel_swizzle) == 1.0
    assert hs.window_reads(kernel_pixel) == 1.0
    assert hs.halo_writes(kernel_swizzle, kernel_pixel) < 1.05          # only the last two columns
    assert hs.halo_writes(lambda hy, hx: hx & 3, hs.rowwise) > 2.0      # the round-2 layout: 2-way
