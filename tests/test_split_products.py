"""The arithmetic of the split products (dpt_mfma_fwd.h split3 / mfma_x6), restated in
numpy: every fp32 value is split exactly into three bf16 parts (round to nearest even,
as v_cvt_pk_bf16_f32), and a K=32 dot product is the sum of the six part products
h*h, h*m, m*h, h*l, l*h, m*m.  Checks, on CPU, that the split is exact up to
2^-24 of the value and that the six-term product stays within fp32 rounding of the
exact (fp64) dot product -- the accuracy claim in DESIGN.md.  The GPU parity tests
(test_gpu_kernels.py) check the kernels themselves against the reference's logits."""
import numpy as np


def bf16_rne(x):
    """fp32 -> bf16 (round to nearest even) -> fp32, bit for bit."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def split3(v):
    v = np.asarray(v, np.float32)
    h = bf16_rne(v)
    r = (v - h).astype(np.float32)  # exact in fp32
    m = bf16_rne(r)
    q = (r - m).astype(np.float32)
    return h, m, bf16_rne(q)


def x6_dot(a, b):
    """sum over k of the six part products, accumulated in fp32 in the kernel's order."""
    ah, am, al = (p.astype(np.float64) for p in split3(a))
    bh, bm, bl = (p.astype(np.float64) for p in split3(b))
    acc = np.float32(0)
    for pa, pb in ((am, bm), (ah, bl), (al, bh), (ah, bm), (am, bh), (ah, bh)):
        acc = np.float32(acc + np.float32((pa * pb).sum()))  # bf16 products are exact
    return acc


def test_split_is_exact_to_2_pow_24():
    rs = np.random.RandomState(0)
    v = (rs.standard_normal(100000) * np.exp(rs.uniform(-20, 20, 100000))).astype(np.float32)
    h, m, l = split3(v)
    resid = v.astype(np.float64) - (h.astype(np.float64) + m + l)
    assert np.all(np.abs(resid) <= 2.0 ** -24 * np.abs(v.astype(np.float64)))
    # the first two residuals are exact fp32 differences
    assert np.array_equal((v - h).astype(np.float32).astype(np.float64), v.astype(np.float64) - h)


def test_six_term_dot_within_fp32_rounding():
    rs = np.random.RandomState(1)
    worst = 0.0
    for _ in range(2000):
        a = rs.standard_normal(32).astype(np.float32)
        b = (rs.standard_normal(32) * 0.05).astype(np.float32)
        exact = float(np.dot(a.astype(np.float64), b.astype(np.float64)))
        scale = float(np.dot(np.abs(a.astype(np.float64)), np.abs(b.astype(np.float64))))
        worst = max(worst, abs(float(x6_dot(a, b)) - exact) / scale)
    # a plain fp32 dot product has error up to ~K * 2^-24 of sum |a||b|; the split form
    # adds the dropped m*l, l*m, l*l terms (< 3 * 2^-24) and six fp32 roundings
    assert worst < 4 * 2.0 ** -24, worst  # measured: 0.8 * 2^-24


def split2_f16(v, e):
    """The MLP's fp16 two-part split (dpt_mfma_fwd.h split2): v x 2^e -> h + m, both fp16
    (round to nearest even), the residual exact in fp32."""
    x = (np.asarray(v, np.float32) * np.float32(2.0 ** e)).astype(np.float32)
    h = x.astype(np.float16).astype(np.float32)
    m = (x - h).astype(np.float32).astype(np.float16).astype(np.float32)
    return h, m


def x3_dot(a, b, ea, eb):
    """h_a m_b + m_a h_b + h_a h_b (exact fp16 products, fp32 accumulation in the kernel's
    order) at scale 2^(ea + eb), scaled back exactly."""
    ah, am = (p.astype(np.float64) for p in split2_f16(a, ea))
    bh, bm = (p.astype(np.float64) for p in split2_f16(b, eb))
    acc = np.float32(0)
    for pa, pb in ((ah, bm), (am, bh), (ah, bh)):
        acc = np.float32(acc + np.float32((pa * pb).sum()))
    return float(acc) * 2.0 ** -(ea + eb)


def test_fp16_two_part_dot_within_fp32_rounding():
    """The MLP's three-product form at the scales dpt_model_create picks for GPT-2-init
    weights (2^12 on |W| < 4, 2^8 on the activations): within a few 2^-24 of sum |a||b|,
    i.e. as accurate as a plain fp32 dot product of that length."""
    rs = np.random.RandomState(2)
    worst = 0.0
    for _ in range(2000):
        a = (rs.standard_normal(32) * np.exp(rs.uniform(-4, 2))).astype(np.float32)  # ln_2 / gelu outputs
        b = (rs.standard_normal(32) * 0.05).astype(np.float32)                       # weights
        exact = float(np.dot(a.astype(np.float64), b.astype(np.float64)))
        scale = float(np.dot(np.abs(a.astype(np.float64)), np.abs(b.astype(np.float64))))
        worst = max(worst, abs(x3_dot(a, b, 8, 12) - exact) / scale)
    assert worst < 8 * 2.0 ** -24, worst  # measured: 1.6 * 2^-24
