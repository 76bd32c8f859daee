"""CPU tests: pin the oracle (oracle/oracle.c) against the golden fixtures and KATs.

The reference cannot run here; the fixtures are float64 SciPy/NumPy
results and closed-form answers derived from the reference's own examples.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, assert_parity, rms_rel_err

GOLD = os.path.join(ROOT, "tests", "golden")


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.mark.parametrize("name", ["fir_c1.npz", "fir_c2.npz", "fir_cc.npz"])
def test_oracle_fir_golden(oracle, name):
    g = load(name)
    f = oracle.Fir(g["taps"], int(g["decim"]), sample_kind=int(np.iscomplexobj(g["x"])))
    y = f.process(g["x"])
    # sequential f32 without FMA vs float64: well inside 1e-5 of RMS
    assert_parity(y, g["y"], 2e-6, name)


def test_oracle_fir_block_invariance(oracle):
    g = load("fir_c2.npz")
    whole = oracle.Fir(g["taps"], 4, sample_kind=1).process(g["x"])
    f = oracle.Fir(g["taps"], 4, sample_kind=1)
    parts, i = [], 0
    for step in (1, 3, 7, 250, 1000, 3, 2931):
        parts.append(f.process(g["x"][i:i + step]))
        i += step
    parts.append(f.process(g["x"][i:]))
    assert np.array_equal(np.concatenate(parts), whole)  # bit-exact: same arithmetic


def test_oracle_fir_impulse_kat(oracle):
    # examples/filter.rs:16-17 pattern: impulse().filter(taps) reproduces the taps exactly
    h = np.linspace(-1, 1, 37).astype(np.float32)
    x = np.zeros(64, np.float32)
    x[0] = 1
    y = oracle.Fir(h, 1, sample_kind=0).process(x)
    assert np.array_equal(y[:37], h) and np.all(y[37:] == 0)


def test_oracle_decimate_phase_kat(oracle):
    # Decimate keeps upstream indices D-1, 2D-1, ... (adapters/mod.rs:30-37)
    x = np.arange(1, 23, dtype=np.float32)
    y = oracle.Fir(np.array([1.0], np.float32), 4, sample_kind=0).process(x)
    assert np.array_equal(y, x[3::4])


def test_oracle_biquad_golden(oracle):
    g = load("biquad.npz")
    rate = float(g["rate"])
    for (kind, f, q), c64, imp in zip(g["designs"], g["coefs"], g["impulse"]):
        c = np.array(oracle.biquad_coefs(int(kind), float(f), float(q), rate))
        # f32 design vs float64: relative to the largest coefficient
        assert np.max(np.abs(c - c64)) <= 2e-6 * np.max(np.abs(c64)) + 1e-7, (kind, c, c64)
        x = np.zeros(256, np.float32)
        x[0] = 1
        y = oracle.biquad_run(int(kind), float(f), float(q), rate, x)
        # recurrence (biquad.rs:43-56) vs float64 lfilter on the SAME f32-designed coefs
        import scipy.signal as ss
        b0, b1, b2, na1, na2 = [float(v) for v in c]
        ref = ss.lfilter([b0, b1, b2], [1.0, -na1, -na2], x.astype(np.float64))
        assert_parity(y, ref, 2e-5, f"biquad kind {kind}")
        # and vs the float64 design (coefficient rounding of the f32 design included)
        assert_parity(y, imp, 2e-4, f"biquad kind {kind} vs f64 design")


def test_oracle_fft_golden(oracle):
    g = load("fft.npz")
    for N in (8, 64, 1024, 4096):
        y = oracle.fft_frame(g[f"x{N}"])
        assert_parity(y, g[f"y{N}"], 1e-6, f"fft N={N}")


def test_oracle_fft_any_n_golden(oracle):
    """Lengths that are not powers of two (rustfft plans any N, src/fft.rs:10-11), odd N's
    collation start -(N/2) included, rfft's drain (fft.rs:35) and a 1000-point STFT."""
    g = load("fft_any.npz")
    for N in g["sizes"]:
        assert_parity(oracle.fft_frame(g[f"x{N}"]), g[f"y{N}"], 1e-6, f"fft N={N}")
    for N in (1001, 14400):
        y = oracle.fft_frame(g[f"rx{N}"].astype(np.complex64))[N // 2:]
        assert_parity(y, g[f"ry{N}"], 1e-6, f"rfft N={N}")
    y = oracle.stft(g["sx"], int(g["sn"]), int(g["shop"]))
    assert y.shape == g["sy"].shape
    assert_parity(y, g["sy"], 1e-6, "stft N=1000")


def test_oracle_fft_tone_kat(oracle):
    # fft(freq(rate, f)) has one bin of magnitude sqrt(N) at f (fft.rs:16 norm)
    N, rate = 1024, 1024.0
    x = oracle.freq(rate, 100.0, 0.0, N)
    y = oracle.fft_frame(x)
    k = np.argmax(np.abs(y))
    assert k == N // 2 + 100
    assert abs(abs(y[k]) - np.sqrt(N)) < 1e-2


def test_oracle_stft_golden(oracle):
    g = load("stft.npz")
    y = oracle.stft(g["x"], int(g["n"]), int(g["hop"]))
    assert y.shape == g["y"].shape
    assert_parity(y, g["y"], 1e-6, "stft")


def test_oracle_pll_kat(oracle):
    # examples/pll.rs / src/main.rs:41-46: a steady tone at f gives output -> f, locked.
    rate, f = 1.8e6, 50e3
    p = oracle.pll_params(0.0, 0.035, rate, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
    x = oracle.freq(rate, f, 0.0, 40000)
    out, locked = oracle.pll_batch(p, x)
    tail = slice(20000, None)
    assert locked[0, tail].all()
    assert abs(out[0, tail].mean() - f) < 0.01 * f


def test_oracle_u8_ingest(oracle):
    iq = np.array([0, 128, 255, 64], np.uint8)
    y = oracle.u8_to_c64(iq)
    assert np.allclose(y, [(-1 + 0j), (127 / 128 - 0.5j)])


def test_rms_metric_sanity():
    a = np.ones(10)
    assert rms_rel_err(a, a) == (0.0, 0.0)


def test_oracle_freq_sweep_shape(oracle):
    """freq_sweep(1.8e6, 20e3, warmup, -200e3..200e3) (examples/pll.rs:8-11): 1/df of
    warmup at the start frequency, then a linear ramp of df^2 Hz/s to the end frequency."""
    f, v = oracle.freq_sweep(1.8e6, 20000.0, True, -200000.0, 200000.0)
    n_warm = round(1.8e6 / 20000.0)
    assert f.size == round((1 / 20000.0 + 400000.0 / 4e8) * 1.8e6)
    assert np.all(f[:n_warm] == -200000.0)
    step = np.diff(f[n_warm:])
    assert np.allclose(step, 4e8 / 1.8e6, rtol=1e-3)
    assert abs(f[-1] - 200000.0) < 250.0
    assert np.allclose(np.abs(v), 1.0, atol=1e-6)


def test_sweep_mirror_matches_oracle(sdr, oracle):
    """sdrgpu.signal.freq_sweep (host source of the mirror) = the oracle's, bit for bit."""
    for args in ((1.8e6, 20000.0, True, -200000.0, 200000.0), (44100.0, 100.0, True, -20000.0, 20000.0),
                 (48000.0, 500.0, False, 3000.0, -3000.0)):
        f, v = oracle.freq_sweep(*args)
        r = sdr.signal.freq_sweep(*args, block=1000).collect()
        assert np.array_equal(r["freq"], f) and np.array_equal(r["value"], v)


def test_freq_mirror_matches_oracle(sdr, oracle):
    x = sdr.signal.freq(1.8e6, 50e3, 0.3, 5000, block=999).collect()
    assert np.array_equal(x, oracle.freq(1.8e6, 50e3, 0.3, 5000))
