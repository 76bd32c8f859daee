"""The Signal mirror (src/signal/mod.rs:13-123): reference pipelines run unchanged.
CPU tests cover the host-only adapters; -m gpu tests run the GPU-backed stages."""
import numpy as np
import pytest

from conftest import assert_parity


def test_decimate_host_only_kat(sdr):
    # Decimate keeps upstream indices wait-1, 2wait-1, ... across block boundaries and
    # keeps reporting the upstream rate (adapters/mod.rs:30-40)
    x = np.arange(103, dtype=np.float32)
    s = sdr.signal.from_array(48000.0, x, block=7).decimate(12000.0)
    assert s.rate() == 48000.0
    assert np.array_equal(s.collect(), x[3::4])


def test_take_skip(sdr):
    x = np.arange(100, dtype=np.float32)
    s = sdr.signal.from_array(10.0, x, block=9).skip(1.5).take(2.0)
    assert np.array_equal(s.collect(), x[15:35])


@pytest.mark.gpu
def test_filter_decimate_fused(sdr, oracle):
    import scipy.signal as ss
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(50000) + 1j * rng.standard_normal(50000)).astype(np.complex64)
    taps = ss.firwin(255, 0.2).astype(np.float32)
    s = sdr.signal.from_array(2.4e6, x, block=4097).filter(taps).decimate(600e3)
    assert s.rate() == 2.4e6
    assert_parity(s.collect(), oracle.Fir(taps, 4, sample_kind=1).process(x))


@pytest.mark.gpu
def test_impulse_filter_kat(sdr):
    taps = np.linspace(-1, 1, 37).astype(np.float32)
    y = sdr.signal.impulse(44100.0, 100).filter(taps).collect()
    assert np.allclose(y[:37], taps, atol=1e-7) and np.all(y[37:] == 0)


@pytest.mark.gpu
def test_window_decimate_map_fft(sdr, oracle):
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(5000) + 1j * rng.standard_normal(5000)).astype(np.complex64)
    n, hop, rate = 256, 128, 1e6
    y = (sdr.signal.from_array(rate, x, block=999).window(n / rate).decimate(rate / hop)
         .map(sdr.signal.fft).collect())
    ref = oracle.stft(x, n, hop)
    assert y.shape == ref.shape
    assert_parity(y, ref)


@pytest.mark.gpu
def test_filter_pll(sdr, oracle):
    f = sdr.filter
    rate = 1.8e6
    x = oracle.freq(rate, 50e3, 0.0, 20000)
    d = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                    f.BiquadD.LowPass(20000.0, 0.7))
    r = sdr.signal.from_array(rate, x, block=3000).filter(d).collect()
    p = oracle.pll_params(0.0, 0.035, rate, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
    ro, rl = oracle.pll_batch(p, x)
    assert np.array_equal(r["value"], ro[0]) and np.array_equal(r["locked"], rl[0].astype(bool))
