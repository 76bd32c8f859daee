"""Sample-rate conversion: resample::SampleRate (src/resample.rs:32-110) over libsamplerate's
sinc / zero-order-hold / linear converters, and the adapters::Resample Signal stage
(src/signal/adapters/resample.rs:17-82).

Sinc converters (ids 0..2): the oracle restates libsamplerate 0.2's src_sinc.c; the
coefficient tables are this project's own (libsamplerate's are absent), so sinc parity is
unpinned against libsamplerate.  The restatement is pinned by an independent closed form
(positions and fixed-point filter indices computed directly, no buffer mechanics: counts,
zero delay, flush), by partition invariance and by tone SNR; GPU vs oracle is bit-exact.

Oracle: oracle_src_* (oracle/oracle.c), a restatement of libsamplerate's samplerate.c /
src_zoh.c / src_linear.c.  libsamplerate itself is a git dependency (Cargo.toml:24-26) that
is not in this image and the reference holds no resampler outputs, so the restatement is
"parity unpinned" against libsamplerate; it is pinned here by known-answer streams (ratio
1 = one-frame delay, 2x linear = midpoints, 1/2 = every other frame) and by block-partition
invariance.  GPU vs oracle: bit-exact (array_equal) outputs and identical frame counts.
"""
import ctypes

import numpy as np
import pytest

LINEAR, ZOH = 4, 3
BEST, MEDIUM, FASTEST = 0, 1, 2


# ----------------------------- CPU: oracle KATs -------------------------------------
def test_oracle_known_answers(oracle):
    x = np.arange(1, 11, dtype=np.float32)
    s = oracle.SampleRate(LINEAR, 1)
    used, y = s.process(1.0, x, 100)
    assert used == 10 and np.array_equal(y.ravel(), np.r_[1, x[:-1]])  # one-frame delay
    used, y = s.process(1.0, x + 10, 100)
    assert np.array_equal(y.ravel(), np.r_[10, x[:-1] + 10])
    s = oracle.SampleRate(LINEAR, 1)
    used, y = s.process(2.0, x, 100)
    assert np.array_equal(y.ravel()[3:], np.arange(1.5, 10, 0.5, dtype=np.float32))
    s = oracle.SampleRate(ZOH, 1)
    used, y = s.process(0.5, x, 100)
    assert np.array_equal(y.ravel(), [1, 2, 4, 6, 8, 10])


@pytest.mark.parametrize("conv", [ZOH, LINEAR], ids=["zoh", "linear"])
@pytest.mark.parametrize("ratio", [48000 * 3.0 / 1.8e6, 0.75, 1.0, 2.5, 48000 / 44100])
def test_oracle_partition_invariance(oracle, conv, ratio):
    """Whole-stream output does not depend on how the input is split into calls."""
    rng = np.random.default_rng(7)
    x = rng.standard_normal((3000, 2)).astype(np.float32)
    a = oracle.SampleRate(conv, 2)
    _, ya = a.process(ratio, x, 100000)
    b = oracle.SampleRate(conv, 2)
    outs, i = [], 0
    while i < x.shape[0]:
        n = int(rng.integers(1, 400))
        used, y = b.process(ratio, x[i:i + n], 100000)
        outs.append(y)
        i += used
    yb = np.concatenate(outs)
    m = min(len(ya), len(yb))
    assert abs(len(ya) - len(yb)) <= 1 and np.array_equal(ya[:m], yb[:m])


def test_oracle_linear_on_a_line(oracle):
    """Linear interpolation of a straight line stays on the line (up to f32 rounding)."""
    x = (0.25 * np.arange(5000)).astype(np.float32)
    s = oracle.SampleRate(LINEAR, 1)
    used, y = s.process(1.37, x, 100000)
    d = np.diff(y.ravel()[2:].astype(np.float64))
    assert np.allclose(d, 0.25 / 1.37, atol=2e-3)


# ----------------------------- CPU: ABI rejections ----------------------------------
def test_src_abi_without_device(sdr):
    L = sdr.lib()
    err = ctypes.c_int(0)
    assert not L.sdrgpu_src_new(0, 9, 1, ctypes.byref(err)) and err.value == 10
    assert not L.sdrgpu_src_new(0, -1, 1, ctypes.byref(err)) and err.value == 10
    assert not L.sdrgpu_src_new(0, 4, 0, ctypes.byref(err)) and err.value == 11
    assert L.sdrgpu_src_get_channels(None) == -2
    assert L.sdrgpu_src_process(None, None) == 2
    assert L.sdrgpu_src_set_ratio(None, 1.0) == 2
    assert L.sdrgpu_src_delete(None) is None
    assert L.sdrgpu_src_strerror(6) == b"SRC ratio outside [1/256, 256] range."
    assert L.sdrgpu_src_strerror(99) is None
    assert L.sdrgpu_src_get_name(4) == b"Linear Interpolator"
    assert L.sdrgpu_src_get_name(5) is None
    from sdrgpu import resample
    assert resample.ConverterType.ZeroOrderHold.name_() == "ZOH Interpolator"
    assert str(resample.Error(16)).startswith("DataOverlap")


# ----------------------------- CPU: sinc restatement ---------------------------------
@pytest.mark.parametrize("conv", [BEST, MEDIUM, FASTEST])
def test_sinc_tables_identical(sdr, oracle, conv):
    """The library's table and the oracle's are the same design, bit for bit; lengths and
    increments are libsamplerate's (2381/340239, 491/22438, 128/2464)."""
    from sdrgpu import resample
    a, ia = resample.sinc_table(conv)
    b, ib = oracle.sinc_table(conv)
    assert ia == ib and a.shape == b.shape and np.array_equal(a, b)
    assert (ia, a.size) == {BEST: (2381, 340239), MEDIUM: (491, 22438), FASTEST: (128, 2464)}[conv]
    assert a[-2:].tolist() == [0.0, 0.0] and a[0] == a.max()
    g = a[0] + 2 * a[ia::ia].astype(np.float64).sum()  # unit DC gain at ratio >= 1
    assert abs(g - 1) < 1e-6


def _sinc_closed_form(c, inc, x, ratio):
    """src_sinc.c's output for a whole mono stream (one call, then end of input) written
    directly: output n sits at input position p_n + f_n (libsamplerate's f64 walk), its
    left taps are x[p_n - j] at filter index start + j*incr, its right taps x[p_n + 1 + j]
    at incr - start + j*incr (fixed point, 12 fraction bits), zeros outside the stream;
    output while p_n + f_n + 1/ratio <= len(x)."""
    fi_inc = inc * min(ratio, 1.0)
    incr = int(np.rint(fi_inc * 4096))
    max_fi = (c.size - 2) << 12
    n = x.size
    xp = np.concatenate([x.astype(np.float64), np.zeros(1)])
    out, p, f = [], 0, 0.0
    while not (p + f + (1.0 / ratio + 1e-20) > n):
        start = int(np.rint(f * fi_inc * 4096))
        outv = 0.0
        for first, sign, base in ((start, -1, p), (incr - start, 1, p + 1)):
            j = np.arange((max_fi - first) // incr + 1)
            fi = first + j * incr
            keep = fi >= 0 if sign < 0 else (fi > 0) | (j == 0)
            fi = fi[keep]
            idx = base + sign * j[keep]
            fr = (fi & 4095) / 4096.0
            ic = c[fi >> 12].astype(np.float64) + fr * (c[(fi >> 12) + 1] - c[fi >> 12]).astype(np.float64)
            vals = np.where((idx >= 0) & (idx < n), xp[np.clip(idx, 0, n)], 0.0)
            outv += float(np.dot(ic, vals))
        out.append(np.float32(outv * fi_inc / inc))
        f += 1.0 / ratio
        r = f - np.rint(f)
        r = r + 1.0 if r < 0 else r
        p += int(np.rint(f - r))
        f = r
    return np.array(out, np.float32)


def _oracle_stream(oracle, conv, ch, ratio, x, block, cap):
    s = oracle.SampleRate(conv, ch)
    outs, i = [], 0
    while True:
        used, y = s.process(ratio, x[i:i + block], cap)
        outs.append(y)
        i += used
        if i >= x.shape[0] and y.shape[0] == 0 and x[i:i + block].shape[0] == 0:
            break
    return np.concatenate(outs)


@pytest.mark.parametrize("conv,ratio", [(FASTEST, 0.08), (FASTEST, 1.0), (FASTEST, 1 / 3),
                                        (FASTEST, 2.5), (MEDIUM, 0.5), (BEST, 48000 / 44100)])
def test_oracle_sinc_closed_form(oracle, conv, ratio):
    rng = np.random.default_rng(21)
    x = rng.standard_normal(2500).astype(np.float32)
    c, inc = oracle.sinc_table(conv)
    ref = _sinc_closed_form(c, inc, x, ratio)
    y = _oracle_stream(oracle, conv, 1, ratio, x.reshape(-1, 1), 4096, 100000).ravel()
    assert y.shape == ref.shape, (y.shape, ref.shape)
    assert np.abs(y - ref).max() <= 1e-6 * np.abs(ref).max()


@pytest.mark.parametrize("ratio", [0.08, 0.75, 1.0, 3.0])
def test_oracle_sinc_partition_invariance(oracle, ratio):
    """Whole-stream output (with the end-of-input flush) is independent of block sizes and
    output capacities, channel by channel identical to mono runs."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((6000, 2)).astype(np.float32)
    a = _oracle_stream(oracle, FASTEST, 2, ratio, x, 100000, 100000)
    b = oracle.SampleRate(FASTEST, 2)
    outs, i = [], 0
    while True:
        n = int(rng.integers(0, 700))
        used, y = b.process(ratio, x[i:i + n], int(rng.integers(1, 900)))
        outs.append(y)
        i += used
        if i >= x.shape[0] and y.shape[0] == 0 and n > 0:
            break
    outs.append(b.process(ratio, x[:0], 100000)[1])
    yb = np.concatenate(outs)
    assert np.array_equal(a, yb)
    m = _oracle_stream(oracle, FASTEST, 1, ratio, x[:, :1].copy(), 100000, 100000)
    assert np.array_equal(a[:, :1], m)


@pytest.mark.parametrize("conv,snr_db", [(FASTEST, 95), (MEDIUM, 115), (BEST, 130)])
def test_oracle_sinc_tone_snr(oracle, conv, snr_db):
    """A passband tone resampled 1.8 Msps -> 144 kHz-like (0.3) and 1.0 matches the
    continuous tone to the table's design attenuation."""
    for ratio in (1.0, 0.3):
        x = np.cos(2 * np.pi * 0.2 * min(ratio, 1) * np.arange(40000)).astype(np.float32)
        y = _oracle_stream(oracle, conv, 1, ratio, x.reshape(-1, 1), 4096, 4096).ravel()
        assert abs(y.size - x.size * ratio) <= 2
        t = np.arange(y.size) / ratio
        ref = np.cos(2 * np.pi * 0.2 * min(ratio, 1) * t)
        m = slice(int(400 / ratio), y.size - int(400 / ratio))
        err = y[m] - ref[m]
        assert 10 * np.log10(np.mean(ref[m] ** 2) / np.mean(err ** 2)) > snr_db, (conv, ratio)


# ----------------------------- GPU parity -------------------------------------------
def _run_both(sdr, oracle, conv, ch, ratio, x, rng, split=True, out_cap=None):
    from sdrgpu import resample
    g = resample.SampleRate(conv, ch)
    o = oracle.SampleRate(conv, ch)
    i, n, stalls = 0, x.shape[0], 0
    gy = []
    while i < n and stalls < 20:
        m = int(rng.integers(1, 700)) if split else n - i
        cap = out_cap if out_cap is not None else int(rng.integers(1, 2000))
        gu, ga = g.process(ratio, x[i:i + m], cap)
        ou, oa = o.process(ratio, x[i:i + m], cap)
        assert gu == ou and ga.shape == oa.shape, (i, m, cap, gu, ou, ga.shape, oa.shape)
        assert np.array_equal(ga, oa), (i, m, cap)
        gy.append(ga)
        i += gu
        stalls = stalls + 1 if gu == 0 and ga.shape[0] == 0 else 0
    assert i >= n
    while True:  # end of input (empty block): nothing (ZOH / linear) or the sinc flush
        gu, ga = g.process(ratio, x[:0], 100)
        ou, oa = o.process(ratio, x[:0], 100)
        assert gu == ou == 0 and np.array_equal(ga, oa)
        gy.append(ga)
        if ga.shape[0] == 0:
            break
        assert conv <= FASTEST
    return g, o, np.concatenate(gy)


@pytest.mark.gpu
@pytest.mark.parametrize("conv", [ZOH, LINEAR], ids=["zoh", "linear"])
@pytest.mark.parametrize("ratio", [1.0, 2.0, 0.5, 48000 * 3.0 / 1.8e6, 48000 / 144000.0,
                                   48000 / 44100, 7.3, 1 / 255.0, 256.0])
@pytest.mark.parametrize("ch", [1, 2, 6])
def test_src_bit_exact(sdr, oracle, conv, ratio, ch):
    rng = np.random.default_rng(int(ratio * 1000) + ch * 7 + conv)
    x = rng.standard_normal((3001, ch)).astype(np.float32)
    _run_both(sdr, oracle, conv, ch, ratio, x, rng)


@pytest.mark.gpu
@pytest.mark.parametrize("conv", [FASTEST, MEDIUM, BEST], ids=["fastest", "medium", "best"])
@pytest.mark.parametrize("ratio", [1.0, 0.5, 48000 * 3.0 / 1.8e6, 1 / 3.0, 48000 / 44100,
                                   2.5, 1 / 255.0, 256.0])
@pytest.mark.parametrize("ch", [1, 2, 3])
def test_src_sinc_bit_exact(sdr, oracle, conv, ratio, ch):
    if conv == BEST and (ratio < 0.01 or ch == 3):
        pytest.skip("covered by the faster converters (same code path, longer table)")
    rng = np.random.default_rng(int(ratio * 1000) + ch * 7 + conv)
    n = 3001 if ratio >= 0.01 else 20000
    x = rng.standard_normal((n, ch)).astype(np.float32)
    _run_both(sdr, oracle, conv, ch, ratio, x, rng)


@pytest.mark.gpu
@pytest.mark.parametrize("ch,ratio", [(100, 48000 * 3.0 / 1.8e6), (64, 2.5), (300, 1 / 200.0),
                                      (1100, 48000 * 3.0 / 1.8e6), (1024, 2.5)])
def test_src_sinc_wide_frames(sdr, oracle, ch, ratio):
    """Wide-frame sinc kernel (>= 64 channels: LDS-staged coefficients, partial channel
    tiles, tap chunks beyond 1024 at ratio 1/200, 1024 / 1100 channels) against the oracle,
    ragged blocks."""
    rng = np.random.default_rng(ch)
    x = rng.standard_normal((2000 if ratio > 0.01 else 6000, ch) if ch < 1000 else (700, ch)).astype(np.float32)
    _run_both(sdr, oracle, FASTEST, ch, ratio, x, rng)


@pytest.mark.gpu
@pytest.mark.parametrize("ch", [96, 1030])
def test_src_sinc_wide_frames_nonfinite(sdr, oracle, ch):
    """Wide-frame sinc kernel with NaN / +-inf samples in a few channels: the frames whose taps
    cover them (and only those) go non-finite, exactly as the restatement does."""
    from sdrgpu import resample
    rng = np.random.default_rng(11)
    x = rng.standard_normal((3000 if ch < 1000 else 900, ch)).astype(np.float32)
    x[700, 5] = np.nan
    x[500, 40] = np.inf
    x[510, 41] = -np.inf
    g = resample.SampleRate(FASTEST, ch)
    o = oracle.SampleRate(FASTEST, ch)
    ratio = 48000 * 3.0 / 1.8e6
    gu, ga = g.process(ratio, x, 1 << 14)
    ou, oa = o.process(ratio, x, 1 << 14)
    assert gu == ou and ga.shape == oa.shape
    np.testing.assert_array_equal(ga, oa)  # NaN == NaN here
    assert np.isnan(ga[:, 5]).any() and np.isfinite(ga[:, 6]).all()
    assert np.isfinite(ga[:, 4]).all() and not np.isfinite(ga[:, 40]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("conv", [ZOH, LINEAR, FASTEST], ids=["zoh", "linear", "sinc"])
def test_src_many_channels_one_shot(sdr, oracle, conv):
    """A batch of 1024 complex streams sharing one ratio = 2048 interleaved channels."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((4096, 2048)).astype(np.float32)
    _run_both(sdr, oracle, conv, 2048, 48000 * 3.0 / 1.8e6 * 7, x, rng, split=False,
              out_cap=1 << 16)


@pytest.mark.gpu
@pytest.mark.parametrize("conv", [ZOH, LINEAR, FASTEST, MEDIUM],
                         ids=["zoh", "linear", "fastest", "medium"])
def test_src_variable_ratio_reset_clone(sdr, oracle, conv):
    from sdrgpu import resample
    rng = np.random.default_rng(11)
    x = rng.standard_normal((6000, 2)).astype(np.float32)
    g = resample.SampleRate(conv, 2)
    o = oracle.SampleRate(conv, 2)
    i = 0
    for step, ratio in enumerate([1.0, 1.3, 0.4, 0.4, 3.0, 0.9]):
        if step == 3:
            assert g.set_ratio(0.7) is None and o.set_ratio(0.7) == 0
        if step == 4:
            g.reset()
            o.reset()
        gu, ga = g.process(ratio, x[i:i + 900], 1500)
        ou, oa = o.process(ratio, x[i:i + 900], 1500)
        assert gu == ou and np.array_equal(ga, oa), step
        i += gu
    # clone carries position, ratio and last_value
    c = g.try_clone()
    gu, ga = c.process(0.9, x[i:i + 500], 2000)
    ou, oa = o.process(0.9, x[i:i + 500], 2000)
    assert gu == ou and np.array_equal(ga, oa)
    assert c.channels() == 2


@pytest.mark.gpu
def test_src_errors_and_empty(sdr):
    from sdrgpu import resample
    L = sdr.lib()
    g = resample.SampleRate(resample.ConverterType.Linear, 1)
    with pytest.raises(resample.Error) as e:
        g.process(300.0, np.ones(10, np.float32), 10)
    assert e.value.code == 6
    with pytest.raises(resample.Error) as e:
        g.set_ratio(1e-3)
    assert e.value.code == 6
    used, y = g.process(1.0, np.zeros(0, np.float32), 10)  # end of input: nothing
    assert used == 0 and y.shape[0] == 0
    buf = np.ones(64, np.float32)  # data_in overlapping data_out
    d = resample.SrcData(buf.ctypes.data, buf.ctypes.data + 16, 8, 8, 0, 0, 0, 1.0)
    assert L.sdrgpu_src_process(g.h, ctypes.byref(d)) == 16


@pytest.mark.gpu
def test_src_process_dev(sdr, oracle):
    from sdrgpu import device, resample
    rng = np.random.default_rng(5)
    x = rng.standard_normal((20000, 2)).astype(np.float32)
    ratio = 48000 / 1.8e6 * 3
    for conv in (LINEAR, FASTEST):
        g = resample.SampleRate(conv, 2)
        o = oracle.SampleRate(conv, 2)
        din = device.DeviceBuffer.from_numpy(x)
        dout = device.DeviceBuffer(8 * 20000)
        used, gen = g.process_dev(ratio, din.ptr, 20000, dout.ptr, 20000)
        g.sync()
        ou, oa = o.process(ratio, x, 20000)
        assert used == ou and gen == oa.shape[0]
        assert np.array_equal(dout.download(gen * 2, np.float32).reshape(-1, 2), oa)


def _adapter_ref(oracle, conv, x, rate_in, rate_out):
    """adapters::Resample's loop (adapters/resample.rs:36-82) on the oracle."""
    o = oracle.SampleRate(conv, 1)
    ratio = float(np.float32(rate_out)) / float(np.float32(rate_in))
    buf, ref, i = np.zeros(0, np.float32), [], 0
    while True:
        take = 4096 - buf.size
        buf = np.concatenate([buf, x[i:i + take]])
        i += min(take, max(0, x.size - i))
        used, out = o.process(ratio, buf, 4096)
        if buf.size == 0 and out.shape[0] == 0:
            break
        buf = buf[used:]
        ref.append(out.ravel())
    return np.concatenate(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("conv", [LINEAR, FASTEST], ids=["linear", "sinc_fastest"])
def test_signal_resample_with_matches_adapter(sdr, oracle, conv):
    """fm.resample_with(SincFastest, 144 kHz) from 1.8 Msps (src/main.rs:50), and Linear."""
    from sdrgpu import resample, signal
    rng = np.random.default_rng(9)
    x = rng.standard_normal(50000).astype(np.float32)
    got = signal.from_array(1.8e6, x, block=7000).resample_with(
        resample.ConverterType(conv), 48000.0 * 3.0)
    assert got.rate() == 144000.0
    assert np.array_equal(got.collect(), _adapter_ref(oracle, conv, x, 1.8e6, 144000.0))


@pytest.mark.gpu
def test_signal_resample_default_best(sdr, oracle):
    """Signal::resample = resample_with(SincBestQuality) (src/signal/mod.rs:78-84), as
    src/main.rs:73 resamples 144 kHz to 48 kHz."""
    from sdrgpu import signal
    rng = np.random.default_rng(10)
    x = rng.standard_normal(30000).astype(np.float32)
    y = signal.from_array(144000.0, x, block=5000).resample(48000.0).collect()
    assert np.array_equal(y, _adapter_ref(oracle, BEST, x, 144000.0, 48000.0))


def test_oracle_resample_golden(oracle):
    """Oracle (serial f64 walk, libsamplerate's form) vs the closed form with exact rational
    positions (tests/golden/make_golden.py): same outputs except where an output's position
    is within 1e-9 of a frame boundary (the walk's rounding may land on either side: ZOH
    then holds the other frame; linear moves by < 1e-5), same counts up to that boundary."""
    import os
    from conftest import ROOT
    d = np.load(os.path.join(ROOT, "tests", "golden", "resample.npz"))
    for i in range(int(d["ncases"])):
        x, ratio = d[f"x{i}"], float(d[f"ratio{i}"])
        for conv, key in ((LINEAR, "lin"), (ZOH, "zoh")):
            used, y = oracle.SampleRate(conv, x.shape[1]).process(ratio, x, 100000)
            ref, amb = d[f"{key}{i}"], d[f"{key}amb{i}"]
            assert abs(len(y) - len(ref)) <= 1 and used >= x.shape[0] - 1, (i, key)
            m = min(len(y), len(ref))
            ok = ~amb[:m]
            if conv == LINEAR:
                assert np.abs(y[:m] - ref[:m]).max() <= 1e-5, (i, key)
            else:
                assert np.array_equal(y[:m][ok], ref[:m][ok]), (i, key)
