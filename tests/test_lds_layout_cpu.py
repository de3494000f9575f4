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


# ds_read_b128's four lane groups (MI355X_MICROARCH.md §LDS): one LDS cycle each when conflict-free
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def test_presplit_weight_reads_are_conflict_free():
    """The three-term fp32 plan's pre-split weight planes (conv3x3_halo_kernel X3 = 2, unet_capi.cpp
    pack3x3_split): 64-byte rows, lane (col, q) reads row col's 16-byte chunk q at position q ^ ((col >> 1) & 3).
    Every ds_read_b128 lane group then touches each of the 64 banks exactly once."""
    for t in range(4):   # the wave's four 16-row groups (row = 16 t + col)
        for g in B128_GROUPS:
            banks = []
            for lane in g:
                col, q = lane & 15, lane >> 4
                r = 16 * t + col
                addr = r * 64 + ((q ^ ((r >> 1) & 3)) << 4)
                banks += [(addr // 4 + i) % 64 for i in range(4)]
            assert sorted(banks) == list(range(64)), (t, g)


def _pix_of(p, tw=16):
    """unet_kernels.hip pix_of_w<TW>: pixel p of a 16 x TW tile -> (row, col), groups of 2 rows x 8 columns."""
    g, j = p >> 4, p & 15
    return 2 * (g // (tw // 8)) + (j >> 3), 8 * (g % (tw // 8)) + (j & 7)


def test_split_once_plane_reads_are_conflict_free_at_every_tap():
    """The split-once three-term kernels: each activation plane holds halo pixel r = hy * HWX + hx as a
    64-byte row, piece q at q ^ ((hy & 1) << 1) -- conv3x3_x3s_kernel (16x16 tiles, HWX = 18, four waves of
    four pixel groups per row group) and conv3x3_x3w_kernel (16x32 tiles, HWX = 34, eight waves).  At every
    tap (dy, dx), for every wave and pixel group, each ds_read_b128 lane group covers the 64 banks once;
    the kernels' per-lane swizzle ((col >> 3) ^ dy) & 1 equals (hy & 1) of the pixel read."""
    for tw, waves in ((16, 4), (32, 8)):
        hwx = tw + 2
        for wp in range(waves):
            for p in range(4):
                for dy in range(3):
                    for dx in range(3):
                        for g in B128_GROUPS:
                            banks = []
                            for lane in g:
                                col, q = lane & 15, lane >> 4
                                py, px = _pix_of((wp * 4 + p) * 16 + col, tw)
                                hy, hx = py + dy, px + dx
                                assert (hy & 1) == (((col >> 3) ^ dy) & 1)
                                addr = (hy * hwx + hx) * 64 + ((q ^ ((hy & 1) << 1)) << 4)
                                banks += [(addr // 4 + i) % 64 for i in range(4)]
                            assert sorted(banks) == list(range(64)), (tw, wp, p, dy, dx, g)


def test_split_once_pass_covers_every_plane_piece_once():
    """The split pass: unit u = (pixel u >> 2, piece u & 3) over the halo's pixels x 4 units writes each
    16-byte piece of each plane exactly once (a permutation of the pieces within every row)."""
    for hwx in (18, 34):
        npix = 18 * hwx
        seen = set()
        for u in range(npix * 4):
            r, pq = u >> 2, u & 3
            hy = r // hwx
            seen.add(r * 64 + ((pq ^ ((hy & 1) << 1)) << 4))
        assert seen == {r * 64 + 16 * k for r in range(npix) for k in range(4)}
