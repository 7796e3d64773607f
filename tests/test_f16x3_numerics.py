"""CPU restatement of the f16x3 GEMM arithmetic (csrc/gemm_x3.hip, f16_mainloop) in numpy: the
split x -> (h, l) = (fp16_rn(x), fp16_rn(2^11 (x - h))), the per-row power-of-two scale of A
from its first 16-wide K-tile, and the three products (64 h_a)(32 h_b) + h_a l_b + l_a h_b
scaled back by 2^-11. Checks the arithmetic's own error claims against float64 — the split is
within 2^-22 relative of x inside the fp16 range, and the three-product GEMM with fp32
accumulation stays at the fp32 GEMM's error level — and the range rules that send a tile to
the x3 fallback. (The GPU test test_gemm_x3_split_accuracy checks the kernel itself.)"""
import numpy as np

F16_LIM_A, F16_LIM_B, F16_TINY = 1023.0, 2047.0, 2.0 ** -13


def split(x):
    x = np.asarray(x, dtype=np.float32)
    h = x.astype(np.float16)
    l = ((x - h.astype(np.float32)) * np.float32(2048.0)).astype(np.float16)
    return h, l


def row_scale(first_tile):
    """2^(8 - e) with max|row| = f 2^e, f in [0.5, 1): the row's max lands in [2^7, 2^8)."""
    m = np.abs(first_tile).max(axis=1)
    _, e = np.frexp(m)
    return np.where(m > 0, np.ldexp(np.float32(1.0), 8 - e), 1.0).astype(np.float32)


def f16x3_gemm(A, B, scale_a=True, bk=16):
    """C = A B with A (M, K), B (K, N) in the f16x3 arithmetic: fp32 accumulation of the three
    fp16 products per 16-deep K-tile (the MFMA's products are exact in fp32)."""
    with np.errstate(over="ignore", invalid="ignore"):   # out-of-range rows overflow fp16
        return _f16x3_gemm(A, B, scale_a, bk)


def _f16x3_gemm(A, B, scale_a, bk):
    A = A.astype(np.float32)
    B = B.astype(np.float32)
    s = row_scale(A[:, :bk]) if scale_a else np.ones(A.shape[0], np.float32)
    As = A * s[:, None]
    ha, la = split(As)
    hb, lb = split(B)
    ha32, la32 = ha.astype(np.float32), la.astype(np.float32)
    hb32, lb32 = hb.astype(np.float32), lb.astype(np.float32)
    acc = np.zeros((A.shape[0], B.shape[1]), np.float32)
    for k0 in range(0, A.shape[1], bk):
        sl = slice(k0, k0 + bk)
        # each product exact in fp64 (11 x 11 bits), summed in fp32 per tile as the accumulator does
        t = ((64 * ha32[:, sl].astype(np.float64)) @ (32 * hb32[sl].astype(np.float64))
             + ha32[:, sl].astype(np.float64) @ lb32[sl].astype(np.float64)
             + la32[:, sl].astype(np.float64) @ hb32[sl].astype(np.float64))
        acc = (acc + t.astype(np.float32)).astype(np.float32)
    in_range = (np.abs(As).max(axis=1) <= F16_LIM_A).all() and (np.abs(B).max(axis=0) <= F16_LIM_B).all()
    return acc * np.float32(2.0 ** -11) / s[:, None], in_range


def test_split_error_bound():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-9, 6.9, 200000))).astype(np.float32)
    x = x[np.abs(x) < 60000]
    h, l = split(x)
    rec = h.astype(np.float64) + l.astype(np.float64) / 2048.0
    big = np.abs(x) >= 2.0 ** -13            # both pieces normal fp16
    rel = np.abs(rec[big] - x[big]) / np.abs(x[big])
    assert rel.max() <= 2.0 ** -22
    assert np.abs(rec - x).max() <= 2.0 ** -35 + 2.0 ** -22 * np.abs(x).max()


def test_three_product_gemm_at_fp32_level():
    rng = np.random.default_rng(2)
    for (M, N, K, amp) in [(64, 48, 1024, 1.0), (40, 30, 300, 1e-6), (40, 30, 70, 30.0)]:
        A = (rng.standard_normal((M, K)) * rng.uniform(0, 1, (M, 1)) * amp).astype(np.float32)
        B = rng.standard_normal((K, N)).astype(np.float32)
        ref = A.astype(np.float64) @ B.astype(np.float64)
        S = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
        C, ok = f16x3_gemm(A, B)
        assert ok
        rel = (np.abs(C - ref) / np.maximum(S, 1e-300)).max()
        # fp32 GEMM (sequential fp32 accumulation) on the same data
        C32 = np.zeros((M, N), np.float32)
        for k0 in range(0, K, 16):
            C32 = (C32 + (A[:, k0:k0 + 16].astype(np.float64)
                          @ B[k0:k0 + 16].astype(np.float64)).astype(np.float32)).astype(np.float32)
        rel32 = (np.abs(C32 - ref) / np.maximum(S, 1e-300)).max()
        assert rel <= max(1.5 * rel32, 2e-7) and rel < 1e-6, (M, N, K, amp, rel, rel32)


def test_range_rules_send_ramping_rows_to_the_fallback():
    """A row scaled from its first K-tile that grows past the fp16 range later is out of range
    (the kernel recomputes that workgroup's tile as x3); a tiny row is scaled into range."""
    rng = np.random.default_rng(3)
    K = 256
    ramp = (rng.standard_normal((8, K)) * np.logspace(-3, 3, K)).astype(np.float32)
    B = rng.standard_normal((K, 8)).astype(np.float32)
    _, ok = f16x3_gemm(ramp, B)
    assert not ok
    tiny = (rng.standard_normal((8, K)) * 1e-7).astype(np.float32)
    _, ok = f16x3_gemm(tiny, B)
    assert ok
    s = row_scale(tiny[:, :16])
    m = np.abs(tiny[:, :16] * s[:, None]).max(axis=1)
    assert ((m >= 128) & (m < 256)).all()
    assert (np.abs(tiny * s[:, None]).max(axis=1) >= F16_TINY).all()
