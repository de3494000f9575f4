"""The three-term fp32 arithmetic of the fp32 plan (csrc/unet_kernels.hip split3_bf16, unet_capi.cpp
split3_host), restated in numpy: x = hi + mid + lo with each term a bf16 (round to nearest
even) and each difference exact in fp32, and a product as the six bf16 products a_i b_j with i + j <= 2.
CPU only: the restatement and the error bounds the plan's fp32 tolerance rests on, not the device code
(the GPU parity tests compare that against the reference at the unchanged fp32 tolerance)."""
import numpy as np


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """fp32 -> the nearest bf16 (ties to even), returned as fp32 (v_cvt_pk_bf16_f32 on finite values)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def split3(x: np.ndarray):
    h = bf16_rne(x)
    r = (x - h).astype(np.float32)
    m = bf16_rne(r)
    l = bf16_rne((r - m).astype(np.float32))
    return h, m, l


def _values(rng, n):
    # fp32 values over the ranges the network's activations and folded weights take (no denormals)
    return (rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n))).astype(np.float32)


def test_split_is_exact():
    """hi + mid + lo equals x exactly, each term is a bf16, and the residual differences are exact in fp32."""
    rng = np.random.default_rng(0)
    x = _values(rng, 200_000)
    h, m, l = split3(x)
    for t in (h, m, l):
        assert np.all((t.view(np.uint32) & 0xFFFF) == 0)          # representable in bf16
    assert np.array_equal(h.astype(np.float64) + m + l, x.astype(np.float64))
    assert np.array_equal((x - h).astype(np.float64), x.astype(np.float64) - h)   # exact difference
    # RNE: |mid| <= ulp_bf16(hi) / 2, so each term is at most 2^-8 of the previous one
    nz = h != 0
    assert np.all(np.abs(m[nz]) <= np.abs(h[nz]) * 2.0 ** -8)


def test_six_products_carry_fp32_accuracy():
    """The dropped terms (i + j >= 3) stay below 2^-24 of |a b| in the worst case: the six-product sum of one
    product is within 2^-23 of the exact product -- inside fp32's own rounding of a single product."""
    rng = np.random.default_rng(1)
    a, b = _values(rng, 200_000), _values(rng, 200_000)
    ta, tb = split3(a), split3(b)
    six = sum(ta[i].astype(np.float64) * tb[j] for i in range(3) for j in range(3) if i + j <= 2)
    exact = a.astype(np.float64) * b
    rel = np.abs(six - exact) / np.abs(exact)
    assert rel.max() < 2.0 ** -23, rel.max()


def test_dot_products_match_fp32_accumulation():
    """A 3x3 layer's K = 9 x Cin dot product: the six-product form with fp32 accumulation (the MFMA's) is as
    close to the fp64 dot product as plain fp32 multiply-add is (3.1e-7 against 2.8e-7 on
    the network)."""
    rng = np.random.default_rng(2)
    k = 9 * 256
    a = rng.standard_normal((512, k)).astype(np.float32)
    b = (rng.standard_normal(k) * 0.05).astype(np.float32)
    exact = a.astype(np.float64) @ b.astype(np.float64)
    ta, tb = split3(a), split3(b)
    acc3 = np.zeros(512, np.float32)
    for i, j in ((1, 1), (2, 0), (0, 2), (1, 0), (0, 1), (0, 0)):   # the kernels' order: small terms first
        acc3 = (acc3 + (ta[i].astype(np.float64) * tb[j]).astype(np.float32).sum(axis=1, dtype=np.float32)).astype(np.float32)
    acc1 = (a * b).sum(axis=1, dtype=np.float32)
    scale = np.abs(exact).max()
    err3 = np.abs(acc3 - exact).max() / scale
    err1 = np.abs(acc1 - exact).max() / scale
    assert err3 < 4 * max(err1, 2.0 ** -24), (err3, err1)
