"""Seeded random parity sweep through the C ABI: shapes the hand-written cases do not name.

Every case draws its shape from a fixed seed (so a failure names a reproducible case id) and
runs the stream as several ragged blocks on ONE handle, so the state carry between calls is
exercised too; the result is compared with the oracle over the whole stream.
  * FIR / FIR-decimate (src/filter/fir.rs:23-32, src/signal/adapters/mod.rs:13-41): sample
    kind f32 / c64 / rtl_tcp u8, real or complex taps, K in 1..300, D in 1..16, every
    algorithm the library exposes (a shape an algorithm does not cover must be refused with
    SDRGPU_ERR_UNSUPPORTED, never computed wrongly);
  * FIR banks (one Fir per channel): nch, K, D, ragged blocks;
  * fft / rfft at random N (src/fft.rs:3-37) against the float64 DFT;
  * PLL (src/filter/pll.rs:48-85) over random block partitions, bit for bit.
Tolerance 1e-5 of RMS, PLL exact."""
import numpy as np
import pytest

from conftest import assert_parity

pytestmark = pytest.mark.gpu

N_FIR = 96
N_BANK = 24
N_FFT = 40
N_PLL = 12


def _blocks(rng, n, kind_bytes_per_sample=1):
    """Random cut points: 1-4 blocks, some of them tiny."""
    k = int(rng.integers(1, 5))
    cuts = sorted(set(int(c) for c in rng.integers(0, n + 1, size=k - 1)))
    return [0] + cuts + [n]


def _fir_case(i):
    rng = np.random.default_rng(1000 + i)
    sk = int(rng.choice([0, 1, 1, 2]))
    tk = int(rng.random() < 0.25)
    K = int(rng.choice([1, 2, 7, 31, 63, 127, 128, 129, 200, 255, 255, 256, 257, 300]))
    D = int(rng.choice([1, 1, 2, 3, 4, 4, 5, 8, 16]))
    n = int(rng.choice([0, 1, 5, 100, 1000, 4097, 20000, 65537, 300001]))
    algo = str(rng.choice(["auto", "auto", "direct", "os", "mx"]))
    return rng, sk, tk, K, D, n, algo


@pytest.mark.parametrize("i", range(N_FIR))
def test_random_fir_stream(sdr, oracle, i):
    from sdrgpu import _lib
    rng, sk, tk, K, D, n, algo = _fir_case(i)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    if tk:
        taps = (taps + 1j * rng.standard_normal(K) / np.sqrt(K)).astype(np.complex64)
    if sk == 2:
        raw = rng.integers(0, 256, size=2 * n, dtype=np.uint8)
        xref = oracle.u8_to_c64(raw)
    elif sk == 1:
        raw = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 0.5).astype(np.complex64)
        xref = raw
    else:
        raw = rng.standard_normal(n).astype(np.float32)
        xref = raw
    a = {"auto": _lib.FIR_AUTO, "direct": _lib.FIR_DIRECT, "os": _lib.FIR_OVERLAP_SAVE,
         "mx": _lib.FIR_MATRIX}[algo]
    # f32 samples x complex taps is not a reference type either: Fir<C, A> needs
    # A: Mul<C, Output = A> (src/filter/convolve.rs:9-13), and f32 * Complex is Complex
    # (include/sdrgpu.h: SDRGPU_ERR_INVALID for that kind pair, any algorithm)
    try:
        f = sdr.filter.Fir(taps, decim=D, sample_kind=sk, algorithm=a).design(2.4e6)
    except _lib.SdrGpuError as e:
        if sk == 0 and tk == 1:
            assert e.code == _lib.ERR_INVALID, e
            return
        assert e.code == _lib.ERR_UNSUPPORTED and algo in ("os", "mx"), e
        pytest.skip(f"{algo} refuses K={K} D={D} sk={sk} tk={tk}")
    assert not (sk == 0 and tk == 1), "f32 samples x complex taps must be refused"
    cuts = _blocks(rng, n)
    outs = []
    for a0, a1 in zip(cuts[:-1], cuts[1:]):
        blk = raw[2 * a0:2 * a1] if sk == 2 else raw[a0:a1]
        try:
            outs.append(f.process(blk))
        except _lib.SdrGpuError as e:
            assert e.code == _lib.ERR_UNSUPPORTED and algo in ("os", "mx"), e
            pytest.skip(f"{algo} refuses this block")
    y = np.concatenate(outs) if outs else np.zeros(0)
    ref = oracle.Fir(taps, D, sample_kind=int(np.iscomplexobj(xref))).process(xref)
    assert y.shape == ref.shape, (y.shape, ref.shape, cuts)
    assert_parity(y, ref, what=f"case {i}: sk={sk} tk={tk} K={K} D={D} n={n} {algo} cuts={cuts}")


@pytest.mark.parametrize("i", range(N_BANK))
def test_random_fir_bank_stream(sdr, oracle, i):
    rng = np.random.default_rng(2000 + i)
    nch = int(rng.choice([1, 2, 3, 17, 64, 129]))
    K = int(rng.choice([15, 63, 127, 255, 255, 271]))
    D = int(rng.choice([1, 1, 2, 4]))
    n = int(rng.choice([256, 1000, 3073, 12000]))
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = ((rng.standard_normal((nch, n)) + 1j * rng.standard_normal((nch, n))) * 0.5).astype(np.complex64)
    bank = sdr.filter.FirBank(taps, nch, sample_kind=sdr.C64, decim=D)
    cuts = _blocks(rng, n)
    outs = [bank.process(x[:, a0:a1]) for a0, a1 in zip(cuts[:-1], cuts[1:]) if a1 > a0]
    y = np.concatenate(outs, axis=1)
    ref = oracle.fir_batch(taps, x, D, nthreads=8)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    for c in range(nch):
        assert_parity(y[c], ref[c], what=f"bank case {i} ch {c}: nch={nch} K={K} D={D} n={n} cuts={cuts}")


@pytest.mark.parametrize("i", range(N_FFT))
def test_random_fft_sizes(sdr, i):
    rng = np.random.default_rng(3000 + i)
    N = int(rng.choice([int(rng.integers(1, 600)), int(rng.integers(600, 5000)),
                        int(2 ** rng.integers(0, 15)), int(rng.integers(5000, 40000))]))
    x = ((rng.standard_normal(N) + 1j * rng.standard_normal(N))).astype(np.complex64)
    X = sdr.fft.fft(x, 1.0)[1]
    # fft.rs:13-23: collated spectrum (start at -(N/2), as numpy's fftshift), 1/sqrt(N)
    ref = np.fft.fftshift(np.fft.fft(x.astype(np.complex128))) / np.sqrt(N)
    assert_parity(X, ref, what=f"fft N={N}")
    xr = rng.standard_normal(N).astype(np.float32)
    R = sdr.fft.rfft(xr, 1.0)[1]
    full = np.fft.fftshift(np.fft.fft(xr.astype(np.complex128))) / np.sqrt(N)
    assert_parity(R, full[N // 2:], what=f"rfft N={N}")


@pytest.mark.parametrize("i", range(N_PLL))
def test_random_pll_partitions_bit_exact(sdr, oracle, i):
    from test_pll_gpu import RATE, fm_channels, main_rs_design, oracle_params
    rng = np.random.default_rng(4000 + i)
    nch = int(rng.choice([1, 5, 64, 65]))
    n = int(rng.choice([1, 37, 1000, 5000]))
    x = fm_channels(rng, nch, n)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    cuts = _blocks(rng, n)
    outs, locks = [], []
    for a0, a1 in zip(cuts[:-1], cuts[1:]):
        if a1 > a0:
            o, l = pll.process(x[:, a0:a1])
            outs.append(o)
            locks.append(l)
    y, lk = np.concatenate(outs, axis=1), np.concatenate(locks, axis=1)
    ref, rl = oracle.pll_batch(oracle_params(oracle), x, nthreads=8)
    assert np.array_equal(lk, rl), f"lock flags, case {i} cuts={cuts}"
    assert np.array_equal(y, ref), f"outputs, case {i} cuts={cuts}"


N_STFT = 12
N_BIQUAD = 12
N_SRC = 16


@pytest.mark.parametrize("i", range(N_STFT))
def test_random_stft_stream(sdr, oracle, i):
    """Window(n) + Decimate(hop) + fft (src/signal/adapters/mod.rs:270-303, 13-41) at random
    (n, hop) over ragged blocks: every frame against the oracle's STFT."""
    rng = np.random.default_rng(5000 + i)
    n = int(rng.choice([int(rng.integers(2, 300)), 256, 1000, 1024, int(rng.integers(300, 3000)), 4096]))
    hop = int(rng.integers(1, 2 * n + 1))
    total = int(rng.integers(0, 6 * n + 3 * hop))
    x = ((rng.standard_normal(total) + 1j * rng.standard_normal(total))).astype(np.complex64)
    s = sdr.fft.Stft(n, hop)
    cuts = _blocks(rng, total)
    parts = [s.process(x[a0:a1]) for a0, a1 in zip(cuts[:-1], cuts[1:])]
    parts = [p for p in parts if p.size]
    ref = oracle.stft(x, n, hop, nthreads=8)
    if not parts:
        assert ref.shape[0] == 0, (n, hop, total)
        return
    y = np.concatenate(parts, axis=0)
    assert y.shape == ref.shape, (y.shape, ref.shape, n, hop, total, cuts)
    for j in range(ref.shape[0]):
        assert_parity(y[j], ref[j], what=f"stft case {i}: n={n} hop={hop} frame {j} cuts={cuts}")


@pytest.mark.parametrize("i", range(N_BIQUAD))
def test_random_biquad_stream_bit_exact(sdr, oracle, i):
    """BiquadD::design + Biquad::apply (src/filter/biquad.rs:25-56,83-155) at random designs,
    sample kinds, channel counts and block partitions: array_equal to the oracle."""
    rng = np.random.default_rng(6000 + i)
    rate = float(rng.choice([48000.0, 144000.0, 1.8e6]))
    kind = str(rng.choice(["LowPass", "HighPass", "BandPass", "Notch", "Lr"]))
    f = sdr.filter
    if kind == "Lr":
        d = f.BiquadD.Lr(float(rng.uniform(10e-6, 200e-6)))
    else:
        d = getattr(f.BiquadD, kind)(float(rng.uniform(0.001, 0.45)) * rate, float(rng.uniform(0.3, 8.0)))
    sk = int(rng.integers(0, 2))
    nch = int(rng.choice([1, 3, 64, 65, 200]))
    n = int(rng.choice([1, 17, 1000, 4001]))
    bq = d.design(rate, sample_kind=sk, nch=nch)
    if sk:
        x = (rng.standard_normal((nch, n)) + 1j * rng.standard_normal((nch, n))).astype(np.complex64)
    else:
        x = rng.standard_normal((nch, n)).astype(np.float32)
    cuts = _blocks(rng, n)
    y = np.concatenate([bq.process(x[:, a0:a1]) for a0, a1 in zip(cuts[:-1], cuts[1:]) if a1 > a0], axis=1)
    c = d.to_c()
    for ch in sorted({0, nch // 2, nch - 1}):
        ref = oracle.biquad_run(c.kind, c.freq, c.q, rate, x[ch])
        np.testing.assert_array_equal(y[ch], ref, err_msg=f"biquad case {i}: {kind} sk={sk} ch {ch} cuts={cuts}")


@pytest.mark.parametrize("i", range(N_SRC))
def test_random_resampler_bit_exact(sdr, oracle, i):
    """SampleRate::process (src/resample.rs:32-110) at random converter, ratio, channel count,
    input block lengths and output capacities, call by call against the oracle (libsamplerate's
    bookkeeping restated; the sinc tables are this library's own)."""
    from test_resample import _run_both
    rng = np.random.default_rng(7000 + i)
    conv = int(rng.choice([0, 1, 2, 3, 4, 2, 4]))
    ratio = float(rng.choice([float(rng.uniform(0.02, 1.0)), float(rng.uniform(1.0, 8.0)),
                              48000 * 3.0 / 1.8e6, 48000 / 144000.0]))
    ch = int(rng.choice([1, 2, 3, 5]))
    n = int(rng.integers(1, 4000))
    x = rng.standard_normal((n, ch)).astype(np.float32)
    _run_both(sdr, oracle, conv, ch, ratio, x, rng)
