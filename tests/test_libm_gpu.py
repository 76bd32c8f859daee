"""GPU parity of the device libm restatements the PLL kernels inline (Pll::apply's arg() and
from_polar, src/filter/pll.rs:72-76 -> f32::atan2 / sin / cos -> glibc atan2f / sinf / cosf on
x86-64 Linux) against glibc itself (oracle.atan2f / oracle.sincosf), bit for bit.

tests/test_libm_restatement.py checks the same header with gcc on the host, where the
device-only code does not exist: the f64 and reciprocal divisions (sdr_fdiv / sdr_fdiv_n) and
the wave ballot that skips atan2f's special-case selects when no lane of a wave needs them.
Here the operands go through sdrgpu_debug_libm, i.e. the same inlined code on the MI355X:
the special-value grid of tests/libm_check.c (zeros, subnormals, +-inf, NaN, 1, huge / tiny
ratios, the |k| = 60 and atanf reduction boundaries), arranged so that some waves hold only
common-path pairs and others mix in one special operand, plus random pairs and both ratio
tails; sincosf over the PLL's phase range and exact multiples of pi/2."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SPECIAL = np.array([0.0, 1.0, 2.0, 0.5, 3.0, 1e-30, 1e30, 1e-45, 1.17549435e-38, 3.4028235e38,
                    np.inf, np.nan, 2.0 ** 60, 2.0 ** 61, 2.0 ** -60, 2.0 ** -61, 2.0 ** 25,
                    2.0 ** -29, 0.4375, 0.6875, 1.1875, 2.4375, 1.0000001, 0.99999994, 7.0, 1e-7],
                   np.float32)


def device_libm(sdr, fn, a, b=None):
    import ctypes
    from sdrgpu import _lib
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b if b is not None else a, np.float32)
    o0, o1 = np.empty_like(a), np.empty_like(a)
    _lib.check(sdr.lib().sdrgpu_debug_libm(0, fn, a.ctypes.data, b.ctypes.data, o0.ctypes.data,
                                           o1.ctypes.data, ctypes.c_size_t(a.size)),
               "sdrgpu_debug_libm")
    return o0, o1


def assert_bits_equal(got, ref, what, args):
    g, r = got.view(np.uint32), ref.view(np.uint32)
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    bad = (g != r) & ~(nan_g & nan_r)
    if bad.any():
        i = np.flatnonzero(bad)[:8]
        detail = ", ".join(f"({', '.join(f'{x[j]!r}' for x in args)}): gpu {got[j]!r} "
                           f"glibc {ref[j]!r}" for j in i)
        raise AssertionError(f"{what}: {bad.sum()} of {got.size} differ: {detail}")


def special_grid():
    """Every ordered pair of SPECIAL values with every sign combination (2704 pairs)."""
    v = SPECIAL
    y, x = np.meshgrid(v, v, indexing="ij")
    ys, xs = [], []
    for s in range(4):
        ys.append((-y if s & 1 else y).ravel())
        xs.append((-x if s & 2 else x).ravel())
    return np.concatenate(ys), np.concatenate(xs)


def test_atan2f_special_grid_mixed_into_common_waves(sdr, oracle):
    rng = np.random.default_rng(72)
    ys, xs = special_grid()
    n_common = 64 * 40
    cy = (rng.standard_normal(n_common) * 10.0 ** rng.uniform(-6, 6, n_common)).astype(np.float32)
    cx = (rng.standard_normal(n_common) * 10.0 ** rng.uniform(-6, 6, n_common)).astype(np.float32)
    # waves of common pairs only (ballot skip), then waves with ONE special pair each, then
    # the dense special grid
    one_y, one_x = cy[:64 * 20].copy(), cx[:64 * 20].copy()
    one_y[::64], one_x[::64] = ys[:20], xs[:20]
    y = np.concatenate([cy, one_y, ys]).astype(np.float32)
    x = np.concatenate([cx, one_x, xs]).astype(np.float32)
    got, _ = device_libm(sdr, 0, y, x)
    assert_bits_equal(got, oracle.atan2f(y, x), "atan2f grid", (y, x))


def test_atan2f_random_and_ratio_tails(sdr, oracle):
    rng = np.random.default_rng(73)
    n = 1 << 20
    bits = rng.integers(0, 2 ** 32, size=(2, n), dtype=np.uint64).astype(np.uint32)
    ya = bits[0].view(np.float32)          # every float pattern: subnormals, inf, NaN included
    xa = bits[1].view(np.float32)
    yb = rng.uniform(-1, 1, n).astype(np.float32)
    xb = rng.uniform(-1, 1, n).astype(np.float32)
    # |y / x| across both atanf tails (2^25 and 2^-29) and the |k| = 60 cut, every sign
    e = rng.integers(-100, 101, n)
    my = (1.0 + rng.integers(0, 1 << 23, n) * 2.0 ** -23).astype(np.float64)
    mx = (1.0 + rng.integers(0, 1 << 23, n) * 2.0 ** -23).astype(np.float64)
    yc = (np.ldexp(my, e // 2 + (e & 1)) * np.where(rng.random(n) < .5, -1, 1)).astype(np.float32)
    xc = (np.ldexp(mx, -(e // 2)) * np.where(rng.random(n) < .5, -1, 1)).astype(np.float32)
    y = np.concatenate([ya, yb, yc])
    x = np.concatenate([xa, xb, xc])
    got, _ = device_libm(sdr, 0, y, x)
    assert_bits_equal(got, oracle.atan2f(y, x), "atan2f random", (y, x))


def test_sincosf_phase_range_and_specials(sdr, oracle):
    rng = np.random.default_rng(74)
    two_pi = np.float32(2 * np.pi)
    a = np.concatenate([
        rng.uniform(-two_pi, two_pi, 1 << 20).astype(np.float32),
        (rng.standard_normal(1 << 16) * 10.0 ** rng.uniform(-45, 0, 1 << 16)).astype(np.float32),
        np.float32(np.pi / 2) * np.arange(-4, 5, dtype=np.float32),
        np.array([0.0, -0.0, 1e-45, -1e-45, 1.17549435e-38, 2.0 ** -12, -(2.0 ** -12), np.nan,
                  0.75, -0.75, 119.9, -119.9], np.float32),
    ]).astype(np.float32)
    s, c = device_libm(sdr, 1, a)
    rs, rc = oracle.sincosf(a)
    assert_bits_equal(s, rs, "sinf", (a,))
    assert_bits_equal(c, rc, "cosf", (a,))
