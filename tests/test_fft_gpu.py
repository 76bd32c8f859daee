"""GPU parity: sdrgpu FFT / rfft / STFT vs the oracle (fft::fft, src/fft.rs:3-37; Window +
Decimate framing, src/signal/adapters/mod.rs:13-41,270-303).  rustfft itself is absent, so
the oracle is the DFT in float64 (parity unpinned at the rustfft-kernel level)."""
import os

import numpy as np
import pytest

from conftest import ROOT, assert_parity

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden")


def cplx(rng, n):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)


@pytest.mark.parametrize("n", [2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096,
                               8192, 16384, 65536, 1 << 18, 1 << 20])
def test_fft_sizes(sdr, oracle, n):
    rng = np.random.default_rng(n)
    count = max(1, min(8, (1 << 16) // n))
    x = cplx(rng, n * count).reshape(count, n)
    y = sdr.fft.FftPlan(n).exec(x)
    for c in range(count):
        assert_parity(y[c], oracle.fft_frame(x[c]), what=f"n={n} frame {c}")


def test_fft_golden(sdr):
    g = np.load(os.path.join(GOLD, "fft.npz"), allow_pickle=False)
    for n in (8, 64, 1024, 4096):
        _, y = sdr.fft.fft(g[f"x{n}"], 1.0)
        assert_parity(y, g[f"y{n}"], what=f"golden {n}")


def test_fft_tone_kat_and_freqs(sdr, oracle):
    n, rate = 1024, 1024.0
    x = oracle.freq(rate, 100.0, 0.0, n)
    f, y = sdr.fft.fft(x, rate)
    k = int(np.argmax(np.abs(y)))
    assert f[k] == 100.0 and abs(abs(y[k]) - np.sqrt(n)) < 1e-2
    assert f[0] == -512.0 and f[-1] == 511.0


def test_rfft(sdr, oracle):
    rng = np.random.default_rng(1)
    for n in (16, 256, 4096):
        x = rng.standard_normal(n).astype(np.float32)
        f, y = sdr.fft.rfft(x, 48000.0)
        ref = oracle.fft_frame(x.astype(np.complex64))[n // 2:]
        assert_parity(y, ref, what=f"rfft {n}")
        assert f[0] == 0.0 and len(f) == n // 2


def test_fft_non_pow2_unsupported(sdr):
    from sdrgpu import _lib
    with pytest.raises(_lib.SdrGpuError) as e:
        sdr.fft.FftPlan(1000)
    assert e.value.code == _lib.ERR_UNSUPPORTED


def test_stft_golden(sdr):
    g = np.load(os.path.join(GOLD, "stft.npz"), allow_pickle=False)
    y = sdr.fft.Stft(int(g["n"]), int(g["hop"])).process(g["x"])
    assert y.shape == g["y"].shape
    assert_parity(y, g["y"], what="stft golden")


@pytest.mark.parametrize("n,hop", [(64, 32), (1024, 512), (4096, 1000), (8192, 4096),
                                   (65536, 32768)])
def test_stft_streaming_chunks(sdr, oracle, n, hop):
    rng = np.random.default_rng(n + hop)
    total = hop * 9 + 123
    x = cplx(rng, total)
    ref = oracle.stft(x, n, hop, nthreads=8)
    s = sdr.fft.Stft(n, hop)
    parts, i = [], 0
    for step in (1, hop - 1, 7, 3 * hop + 5, hop // 2):
        parts.append(s.process(x[i:i + step]))
        i += step
    parts.append(s.process(x[i:]))
    y = np.concatenate([p for p in parts if p.size], axis=0)
    assert y.shape == ref.shape
    for j in range(ref.shape[0]):
        assert_parity(y[j], ref[j], what=f"n={n} hop={hop} frame {j}")


def test_stft_c3_shape_device(sdr, oracle):
    """configs[2] shape (64k-point frames, 50 % overlap) on device buffers, 24 frames."""
    from sdrgpu.device import DeviceBuffer
    n, hop = 65536, 32768
    rng = np.random.default_rng(3)
    total = hop * 24
    x = cplx(rng, total)
    s = sdr.fft.Stft(n, hop)
    nf = s.output_len(total)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nf * n)
    assert s.process_dev(dx.ptr, total, dy.ptr, nf) == nf
    s.sync()
    y = dy.download().reshape(nf, n)
    for j in (0, 1, 11, nf - 1):
        ref = oracle.stft(x[:(j + 1) * hop], n, hop)[j]
        assert_parity(y[j], ref, what=f"frame {j}")
