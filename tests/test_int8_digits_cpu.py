"""CPU model of the int8-MFMA u8 FIR arithmetic (unnamed-rust-sdr_amd/csrc/fir_mxi.hip).

The kernel computes RtlTcpSignal::next -> Fir::apply -> Decimate (reference
src/rtltcp.rs:156-164, src/filter/fir.rs:23-32, src/signal/adapters/mod.rs:30-37) as
  t = rint(h 2^S), S = tap_scale_exp + 7, tap_scale_exp = 15 - exponent(max |h|)
  t = 2^16 d2 + 2^8 d1 + d0, d_i balanced int8 digits
  C_i = sum_k d_i[k] (code - 128)    exact in i32 (v_mfma_i32_16x16x64_i8)
  y = fma(C2, 2^(16-S-7), fma(C1, 2^(8-S-7), C0 2^(-S-7)))   in f32
This file restates those steps in numpy (the digit split, the i32 bounds, the f32 combine) and
checks them against the oracle's FIR on the same codes, so the arithmetic is pinned on the CPU;
tests/test_ingest_gpu.py checks the kernel itself against the same oracle."""
import numpy as np
import pytest


def tap_scale_exp(taps):
    # fir_mfma.hip fir_mx_prepare: 15 - e, max|h| = m 2^e, m in [0.5, 1)
    hmax = float(np.max(np.abs(taps)))
    return min(126, max(-126, 15 - np.frexp(np.float32(hmax))[1]))


def digits(taps):
    S = tap_scale_exp(taps) + 7
    t = np.rint(taps.astype(np.float32) * np.float32(2.0 ** S)).astype(np.int64)
    d0 = ((t + 128) & 255) - 128
    t1 = (t - d0) >> 8
    d1 = ((t1 + 128) & 255) - 128
    d2 = (t1 - d1) >> 8
    return S, t, d0, d1, d2


def model_fir_u8(taps, raw, D=4):
    """The kernel's arithmetic, output m = sum_k h[k] x[4m + 3 - k] (zero history)."""
    S, t, d0, d1, d2 = digits(taps)
    K = taps.size
    x = raw.astype(np.int64).reshape(-1, 2) - 128          # (code - 128): exact int8
    n = x.shape[0]
    xp = np.concatenate([np.zeros((K - 1, 2), np.int64), x])
    m = np.arange(D - 1, n, D)
    out = np.empty((m.size, 2), np.float32)
    sc0 = np.float32(2.0 ** (-(S + 7)))
    sc1, sc2 = np.float32(sc0 * 256), np.float32(sc0 * 65536)
    for comp in range(2):
        C = []
        for d in (d0, d1, d2):
            # C[m] = sum_k d[k] x[m - k], exact integers
            acc = np.zeros(m.size, np.int64)
            for k in range(K):
                acc += d[k] * xp[m + K - 1 - k, comp]
            assert np.abs(acc).max(initial=0) < 2 ** 31  # i32 accumulators never wrap
            C.append(acc)
        c0, c1, c2 = (np.float32(c) for c in C)
        inner = (c1.astype(np.float64) * sc1 + np.float32(c0 * sc0)).astype(np.float32)  # fma: one rounding
        out[:, comp] = (c2.astype(np.float64) * sc2 + inner).astype(np.float32)
    return out[:, 0] + 1j * out[:, 1]


@pytest.mark.parametrize("scale", [1e-20, 1.0, 3e7])
def test_digit_split_is_exact_and_in_range(scale):
    rng = np.random.default_rng(11)
    taps = (rng.standard_normal(255) * scale).astype(np.float32)
    S, t, d0, d1, d2 = digits(taps)
    assert np.abs(t).max() <= 2 ** 22                       # |h| 2^S < 2^22 (rounding may reach it)
    for d in (d0, d1, d2):
        assert d.min() >= -128 and d.max() <= 127           # balanced int8 digits
    np.testing.assert_array_equal((d2 << 16) + (d1 << 8) + d0, t)
    # the taps' only rounding: to integers |t| <= 2^22, i.e. <= 2^-22 of max |h|
    rel = np.abs(t * 2.0 ** -S - taps.astype(np.float64)).max() / np.abs(taps).max()
    assert rel <= 2.0 ** -22


def test_worst_case_accumulators_fit_i32():
    """|C| <= 5 chunks x 64 x 128 x 128 < 2^23 per digit plane (the kernel's K = 320 window)."""
    assert 5 * 64 * 128 * 128 < 2 ** 31
    taps = np.full(257, -1.0, np.float32)   # all digits at their extremes, K = 257
    raw = np.zeros(2 * 2000, np.uint8)       # code 0 -> -128: every product at its maximum
    y = model_fir_u8(taps, raw)
    assert np.isfinite(y).all()


def test_model_matches_the_oracle_fir(oracle):
    """The int8 arithmetic restated here meets the parity tolerance against the oracle's f32
    FIR on the converted codes (the kernel's only approximation is the taps' rounding to integers)."""
    from conftest import assert_parity
    import scipy.signal as ss
    rng = np.random.default_rng(5)
    for taps in (ss.firwin(255, 0.2).astype(np.float32),
                 (rng.standard_normal(97) / 10).astype(np.float32)):
        raw = rng.integers(0, 256, size=2 * 6000, dtype=np.uint8)
        ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
        y = model_fir_u8(taps, raw)
        assert_parity(y, ref, tol=2e-6, what=f"K {taps.size}")


@pytest.fixture(scope="module")
def oracle():
    import pyoracle
    return pyoracle
