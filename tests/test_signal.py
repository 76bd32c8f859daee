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


# ---- rtl_tcp byte blocks (CU8): adapters count SAMPLES (byte pairs), never single bytes ----
def _iq(n, seed=0):
    return np.random.default_rng(seed).integers(0, 256, 2 * n, dtype=np.uint8)


def test_cu8_take_skip_decimate_count_samples(sdr, oracle):
    from sdrgpu import _lib
    iq = _iq(1000)
    s = sdr.signal.from_array(100.0, iq, block=37, sample_kind=_lib.CU8)
    x = oracle.u8_to_c64(iq)
    got = s.skip(1.5).take(2.0).collect()          # samples 150 .. 350 -> bytes 300 .. 700
    assert got.dtype == np.complex64 and np.array_equal(got, x[150:350])
    d = sdr.signal.from_array(100.0, iq, block=37, sample_kind=_lib.CU8).decimate(25.0).collect()
    assert np.array_equal(d, x[3::4])                # kept samples wait-1, 2wait-1, ...
    # iter and map hand Complex<f32> samples to user code, as RtlTcpSignal::next does
    it = list(sdr.signal.from_array(100.0, iq, block=37, sample_kind=_lib.CU8).iter())
    assert np.array_equal(np.array(it, np.complex64), x)
    m = sdr.signal.from_array(100.0, iq, block=37, sample_kind=_lib.CU8).map(lambda b: b * 2)
    assert np.array_equal(m.collect(), x * np.float32(2))


def test_as_usize_rounds_the_f32_value():
    """FreqSweep::new's `(t * rate).round() as usize` (sources.rs:133-134) on f32 values at
    and above 2^23 and just below one half (advisor finding: f32 rounding of |v| + 0.5)."""
    from sdrgpu.signal import _as_usize
    f32 = np.float32
    assert _as_usize(f32(2 ** 23 + 1)) == 2 ** 23 + 1
    assert _as_usize(f32(2 ** 24 + 2)) == 2 ** 24 + 2
    assert _as_usize(f32(0.49999997)) == 0
    assert _as_usize(f32(0.5)) == 1 and _as_usize(f32(1.5)) == 2 and _as_usize(f32(2.5)) == 3
    assert _as_usize(f32(-3.7)) == 0 and _as_usize(f32(0.0)) == 0
    assert _as_usize(f32(8388609.0) * f32(1.0)) == 8388609


def test_as_usize_saturates_like_rust_as():
    """Rust's `f32 as usize` saturates: NaN -> 0, -inf -> 0, +inf -> usize::MAX (advisor
    finding r3); freq_sweep with df = 0 and rate = 0 (inf * 0 = NaN) is an empty sweep."""
    import warnings
    from sdrgpu import _lib
    from sdrgpu.signal import USIZE_MAX, _as_usize, freq_sweep
    f32 = np.float32
    assert _as_usize(f32(np.nan)) == 0 and _as_usize(f32(-np.inf)) == 0
    assert _as_usize(f32(np.inf)) == USIZE_MAX == 2 ** 64 - 1
    assert _as_usize(f32(3.0e38)) == USIZE_MAX and _as_usize(f32(2.0 ** 40)) == 2 ** 40
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        assert freq_sweep(0.0, 0.0, True, 0.0, 10.0).collect().size == 0
        with pytest.raises(_lib.SdrGpuError):
            freq_sweep(np.inf, 1.0, False, 0.0, 10.0)   # +inf samples: refused, not materialised


def test_cu8_window_raw_frames_convert_samples(sdr, oracle):
    """window(..).decimate(..).map(f) with a non-FFT map sees Complex samples, as
    RtlTcpSignal::next yields them (src/rtltcp.rs:156-164)."""
    from sdrgpu import _lib
    iq = _iq(300, 1)
    n, hop = 16, 8
    fr = (sdr.signal.from_array(1.0, iq, block=50, sample_kind=_lib.CU8).window(n / 1.0)
          .decimate(1.0 / hop).map(lambda f: f).collect())
    x = oracle.u8_to_c64(iq)
    assert fr.shape == (300 // hop, n)
    for j in range(fr.shape[0]):
        beg = (j + 1) * hop - n
        want = np.zeros(n, np.complex64)
        want[max(0, -beg):] = x[max(0, beg):beg + n]
        assert np.array_equal(fr[j], want)


@pytest.mark.gpu
def test_cu8_filter_then_pll_and_fir_chain(sdr, oracle):
    """rtl.listen().filter(taps).filter(pll) and a two-FIR chain: the FIR after CU8 input
    yields C64 samples, which the next stage must consume as C64 (advisor finding)."""
    from sdrgpu import _lib
    import scipy.signal as ss
    f = sdr.filter
    rate = 1.8e6
    iq = _iq(30000, 2)
    x = oracle.u8_to_c64(iq)
    taps = ss.firwin(63, 0.3).astype(np.float32)
    taps2 = ss.firwin(31, 0.4).astype(np.float32)
    d = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                    f.BiquadD.LowPass(20000.0, 0.7))
    src = lambda: sdr.signal.from_array(rate, iq, block=4096, sample_kind=_lib.CU8)
    r = src().filter(taps).filter(d).collect()
    y1 = oracle.Fir(taps, 1, sample_kind=1).process(x)
    p = oracle.pll_params(0.0, 0.035, rate, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
    # the PLL is bit-exact to the oracle fed the same FIR output: the u8 FIR stage's own
    # (the int8 kernel's; within tolerance of the oracle FIR, not bit-equal to the c64 path)
    yg = src().filter(taps).collect()
    assert_parity(yg, y1)
    ro, rl = oracle.pll_batch(p, yg)
    assert np.array_equal(r["value"], ro[0]) and np.array_equal(r["locked"], rl[0].astype(bool))
    chain = src().filter(taps).filter(taps2).collect()
    assert chain.dtype == np.complex64
    assert_parity(chain, oracle.Fir(taps2, 1, sample_kind=1).process(y1))


@pytest.mark.gpu
def test_cu8_window_decimate_map_fft(sdr, oracle):
    """examples/live.rs:29-39: rtl.listen().window(..).decimate(fps).map(fft) -- the raw bytes
    go to the GPU STFT (u8 frame load) and equal the oracle STFT of the converted samples."""
    from sdrgpu import _lib
    iq = _iq(6000, 3)
    n, hop, rate = 1000, 400, 1e6
    y = (sdr.signal.from_array(rate, iq, block=777, sample_kind=_lib.CU8).window(n / rate)
         .decimate(rate / hop).map(sdr.signal.fft).collect())
    ref = oracle.stft(oracle.u8_to_c64(iq), n, hop)
    assert y.shape == ref.shape
    assert_parity(y, ref)


@pytest.mark.gpu
def test_cu8_resample_with_matches_c64_path(sdr, oracle):
    """resample_with on rtl_tcp bytes converts them as RtlTcpSignal::next does and labels the
    output Complex<f32>: equal to the same stage fed the converted samples (advisor finding)."""
    from sdrgpu import _lib
    from sdrgpu.resample import ConverterType
    iq = _iq(20000, 4)
    x = oracle.u8_to_c64(iq)
    rate = 1.8e6
    a = sdr.signal.from_array(rate, iq, block=3000, sample_kind=_lib.CU8).resample_with(
        ConverterType.Linear, 144e3)
    b = sdr.signal.from_array(rate, x, block=3000).resample_with(ConverterType.Linear, 144e3)
    assert a.sample_kind == _lib.C64
    ya, yb = a.collect(), b.collect()
    assert ya.dtype == np.complex64 and np.array_equal(ya, yb)
    # a following decimate counts Complex samples, not byte pairs
    d = sdr.signal.from_array(rate, iq, block=3000, sample_kind=_lib.CU8).resample_with(
        ConverterType.Linear, 144e3).decimate(72e3).collect()
    assert np.array_equal(d, yb[1::2])


def test_fm_receiver_designs_host_only(sdr):
    """sdrgpu.fm mirrors src/main.rs:41-60's designs and refuses input that is not rtl_tcp
    bytes (host logic only; the chain itself runs in tests/test_fm_chain_gpu.py)."""
    from sdrgpu import _lib, fm
    from sdrgpu.signal import from_array
    d = fm.discriminator_design()
    assert (d.reference, d.gain) == (0.0, 0.035)
    p = fm.pilot_design()
    assert (p.reference, p.gain) == (19000.0, 0.0002)
    # BiquadD::Lr(1.0 / (75.0 * 0.001 * 0.001)) evaluated in f32, as the reference's literals are
    dr = np.float32(1.0) / (np.float32(75.0) * np.float32(0.001) * np.float32(0.001))
    assert np.float32(fm.deemphasis().freq) == dr and fm.deemphasis().kind == _lib.BQ_LR
    with pytest.raises(_lib.SdrGpuError):
        fm.receiver(from_array(1.8e6, np.zeros(16, np.complex64)))
