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
        assert f[0] == 0.0 and len(f) == n - n // 2


# lengths that are not powers of two: mixed-radix tiles (smooth, <= 4096), mixed-radix
# four-step (smooth, > 4096) and Bluestein (a prime factor > 13)
ANY_N = [1, 3, 5, 6, 7, 9, 12, 17, 100, 1000, 1001, 1009, 1331, 2187, 3000, 4095, 4099,
         6561, 12288, 14400, 15625, 30030, 65537, 100000, 262139]


@pytest.mark.parametrize("n", ANY_N)
def test_fft_any_size(sdr, oracle, n):
    rng = np.random.default_rng(n + 7)
    count = max(1, min(5, 20000 // n))
    x = cplx(rng, n * count).reshape(count, n)
    y = sdr.fft.FftPlan(n).exec(x)
    for c in range(count if n <= 20000 else 1):
        ref = oracle.fft_frame(x[c]) if n <= 20000 else \
            (np.fft.fftshift(np.fft.fft(x[c].astype(np.complex128))) / np.sqrt(n))
        assert_parity(y[c], ref, what=f"n={n} frame {c}")


def test_fft_any_golden(sdr):
    """examples/live.rs:30's 1000-point and examples/fft.rs:64,78's 14,400-point transforms
    (and 1001, primes, 6, 12288) against NumPy float64 fixtures."""
    g = np.load(os.path.join(GOLD, "fft_any.npz"), allow_pickle=False)
    for n in g["sizes"]:
        _, y = sdr.fft.fft(g[f"x{n}"], 1.0)
        assert_parity(y, g[f"y{n}"], what=f"golden fft {n}")
    for n in (1001, 14400):
        f, y = sdr.fft.rfft(g[f"rx{n}"], 144000.0)
        assert y.shape == (n - n // 2,) and f.shape == y.shape
        assert_parity(y, g[f"ry{n}"], what=f"golden rfft {n}")
    y = sdr.fft.Stft(int(g["sn"]), int(g["shop"])).process(g["sx"])
    assert_parity(y, g["sy"], what="golden stft 1000")


def test_rfft_device_pointers_match_host_path(sdr):
    """sdrgpu_rfft_exec_dev (device-resident frames, the examples/fft.rs batch shape) gives
    exactly the host-pointer rfft's values."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(5)
    for n, count in ((14400, 7), (1000, 33), (4096, 3)):
        x = rng.standard_normal((count, n)).astype(np.float32)
        p = sdr.fft.FftPlan(n)
        ref = p.exec_real(x)
        dx = DeviceBuffer.from_numpy(x)
        dy = DeviceBuffer.empty(count * (n - n // 2), np.complex64)
        p.exec_real_dev(dx.ptr, dy.ptr, count)
        p.sync()
        assert np.array_equal(dy.download().reshape(count, n - n // 2), ref)


@pytest.mark.parametrize("n", [1000, 1001, 14400, 4099, 65536])
def test_rfft_any_size(sdr, oracle, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal((3, n)).astype(np.float32)
    y = sdr.fft.FftPlan(n).exec_real(x)
    assert y.shape == (3, n - n // 2)
    for c in range(3):
        ref = np.fft.fftshift(np.fft.fft(x[c].astype(np.complex128)))[n // 2:] / np.sqrt(n)
        assert_parity(y[c], ref, what=f"rfft n={n} frame {c}")


def test_rfft_14400_packed_batch_and_unaligned(sdr):
    """examples/fft.rs's 14,400-point rfft runs as a packed 7,200-point complex transform
    (two frames per workgroup): an odd frame count against NumPy f64, and a 4-byte-offset
    input (not c64-aligned: the full 14,400-point kernel takes it) agreeing within parity."""
    from sdrgpu.device import DeviceBuffer
    n, count = 14400, 65
    rng = np.random.default_rng(14400)
    x = rng.standard_normal((count, n)).astype(np.float32)
    x[3] = 0.0
    x[4, 17] = 1.0  # impulse: flat spectrum
    p = sdr.fft.FftPlan(n)
    y = p.exec_real(x)
    for c in (0, 3, 4, 31, count - 1):
        ref = np.fft.fftshift(np.fft.fft(x[c].astype(np.complex128)))[n // 2:] / np.sqrt(n)
        if c == 3:
            assert np.all(y[c] == 0)
        else:
            assert_parity(y[c], ref, what=f"packed rfft frame {c}")
    raw = DeviceBuffer.from_numpy(np.concatenate([np.zeros(1, np.float32), x[:5].ravel()]))
    dy = DeviceBuffer.empty(5 * (n - n // 2), np.complex64)
    p.exec_real_dev(raw.ptr + 4, dy.ptr, 5)
    p.sync()
    yu = dy.download().reshape(5, n - n // 2)
    for c in range(5):
        if c == 3:
            assert np.all(yu[c] == 0)
        else:
            assert_parity(yu[c], y[c].astype(np.complex128), what=f"unaligned rfft frame {c}")


@pytest.mark.parametrize("n,hop", [(1000, 400), (1000, 1000), (1001, 333), (14400, 7200),
                                   (4099, 2048), (64, 100), (1000, 2500), (4096, 5000), (16, 1),
                                   (65536, 70000)])
def test_stft_any_size_streaming(sdr, oracle, n, hop):
    """Window(n) + Decimate(hop) streamed in ragged blocks (adapters/mod.rs:270-303), including
    hops longer than the frame (frames skip samples) and hop = 1 (a frame per sample)."""
    rng = np.random.default_rng(n * 3 + hop)
    total = hop * 7 + 55
    x = cplx(rng, total)
    ref = oracle.stft(x, n, hop, nthreads=8)
    s = sdr.fft.Stft(n, hop)
    parts, i = [], 0
    for step in (1, hop - 1, 5, 2 * hop + 3):
        parts.append(s.process(x[i:i + step]))
        i += step
    parts.append(s.process(x[i:]))
    y = np.concatenate([p for p in parts if p.size], axis=0)
    assert y.shape == ref.shape
    for j in range(ref.shape[0]):
        assert_parity(y[j], ref[j], what=f"n={n} hop={hop} frame {j}")


def test_fft_many_frames_batching(sdr, oracle):
    """Enough frames that the four-step / Bluestein plans run several scratch batches."""
    from sdrgpu.device import DeviceBuffer
    for n, count in ((14400, 2400), (4099, 4500)):
        rng = np.random.default_rng(n)
        x = cplx(rng, n * count)
        p = sdr.fft.FftPlan(n)
        dx = DeviceBuffer.from_numpy(x)
        dy = DeviceBuffer.empty(n * count)
        p.exec_dev(dx.ptr, dy.ptr, count)
        p.sync()
        for c in (0, count // 2, count - 1):
            y = dy.download(n, offset_bytes=8 * n * c)
            assert_parity(y, oracle.fft_frame(x[c * n:(c + 1) * n]), what=f"n={n} frame {c}")


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


C3_FRAMES = 700   # > 2 x 256: three scratch batches over both streams (fft.hip launch loop)
C3_CHECK = (0, 1, 255, 256, 257, 511, 512, 513, C3_FRAMES - 2, C3_FRAMES - 1)


def _c3_frame_span(x, j, n, hop):
    """Stream samples of STFT frame j: [(j+1)hop - n, (j+1)hop), zeros before 0
    (Window zero prefill, src/signal/adapters/mod.rs:277-299)."""
    beg = (j + 1) * hop - n
    if beg >= 0:
        return x[beg:beg + n]
    return np.concatenate([np.zeros(-beg, x.dtype), x[:beg + n]])


@pytest.mark.parametrize("mode", ["c64", "db", "u8"])
def test_stft_c3_multibatch_schedule(sdr, oracle, mode):
    """configs[2] exactly as bench_configs.py times it: Stft(65536, 32768).process_dev over
    700 frames in ONE call, so the 64K four-step runs its two-stream multi-batch schedule
    (batches of 256 frames alternating between the caller's stream and the plan's aux stream,
    each with its own half of the scratch slab, joined by events).  Frames at every batch
    boundary, both streams and the tail are checked against the oracle FFT of the frame's own
    span (fft.rs:3-28 + Window/Decimate framing), for the c64 store, the fused dB store
    (complexseries.rs:90-92) and rtl_tcp u8 input (rtltcp.rs:156-164)."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    n, hop = 65536, 32768
    total = hop * C3_FRAMES
    rng = np.random.default_rng(700)
    if mode == "u8":
        iq = rng.integers(0, 256, 2 * total, dtype=np.uint8)
        x = oracle.u8_to_c64(iq)
        s = sdr.fft.Stft(n, hop, input_kind=_lib.CU8)
        dx = DeviceBuffer.from_numpy(iq)
    else:
        x = cplx(rng, total)
        s = sdr.fft.Stft(n, hop, output="db" if mode == "db" else "complex")
        dx = DeviceBuffer.from_numpy(x)
    nf = s.output_len(total)
    assert nf == C3_FRAMES
    obytes = 4 if mode == "db" else 8
    dy = DeviceBuffer.empty(nf * n * obytes // 8 + 1)
    assert s.process_dev(dx.ptr, total, dy.ptr, nf) == nf
    s.sync()
    for j in C3_CHECK:
        ref = oracle.fft_frame(_c3_frame_span(x, j, n, hop))
        if mode == "db":
            y = dy.download(n, dtype=np.float32, offset_bytes=4 * n * j)
            _check_db(y, ref, f"c3 db frame {j}")
        else:
            y = dy.download(n, offset_bytes=8 * n * j)
            assert_parity(y, ref, what=f"c3 {mode} frame {j}")
    # the stream state after the call: the next call's first frame continues the stream
    if mode == "c64":
        extra = cplx(rng, hop)
        y2 = s.process(extra)
        ref = oracle.fft_frame(np.concatenate([x[-(n - hop):], extra]))
        assert y2.shape == (1, n)
        assert_parity(y2[0], ref, what="c3 next-call frame")


@pytest.mark.parametrize("nframes", [1, 2, 3, 9, 17, 64])
def test_stft_64k_small_blocks(sdr, oracle, nframes):
    """64K STFT blocks of 1-64 frames (one partial scratch batch, fewer workgroups than
    CUs, the stream-start history frame included): every frame against the oracle."""
    from sdrgpu.device import DeviceBuffer
    n, hop = 65536, 32768
    total = hop * nframes
    rng = np.random.default_rng(nframes)
    x = cplx(rng, total)
    s = sdr.fft.Stft(n, hop)
    nf = s.output_len(total)
    assert nf == nframes
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nf * n)
    assert s.process_dev(dx.ptr, total, dy.ptr, nf) == nf
    s.sync()
    for j in range(nf):
        y = dy.download(n, offset_bytes=8 * n * j)
        assert_parity(y, oracle.fft_frame(_c3_frame_span(x, j, n, hop)), what=f"frame {j}")


def test_stft_64k_repeat_bit_identical(sdr):
    """The same 300-frame block through fresh 64K STFT handles 6 times back to back (warm
    caches, scratch slab reused across the two-stream batches): every output word of every
    run must equal the first run's (the four-step is deterministic whatever workgroup runs a
    piece), and the first run's frames match NumPy."""
    from sdrgpu.device import DeviceBuffer
    n, hop, nfr = 65536, 32768, 300
    total = hop * nfr
    rng = np.random.default_rng(11)
    x = cplx(rng, total)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nfr * n)
    first = None
    for rep in range(6):
        s = sdr.fft.Stft(n, hop)
        assert s.process_dev(dx.ptr, total, dy.ptr, nfr) == nfr
        s.sync()
        y = dy.download(nfr * n)
        if first is None:
            first = y
            for j in (0, 1, 150, nfr - 1):
                span = _c3_frame_span(x, j, n, hop).astype(np.complex128)
                ref = np.fft.fftshift(np.fft.fft(span)) / np.sqrt(n)
                assert_parity(y[j * n:(j + 1) * n], ref, what=f"frame {j}")
        else:
            assert np.array_equal(y.view(np.uint64), first.view(np.uint64)), f"run {rep} differs"
        s.close()


def test_stft_64k_dynamic_range_and_nan(sdr, oracle):
    """configs[2]'s 64K four-step at whole-stream scales from 1e-30 to 1e30, with an all-zero
    frame and a strong tone over a 1e-6 noise floor (120 dB of range in every frame), against
    the float64 DFT.  A tone's spectrum is one peak ~sqrt(N) = 256 times the bins' RMS, so any
    f32 FFT (rustfft's included) rounds that bin at ~1e-7 of the PEAK, i.e. 2-4e-5 of the RMS
    (profiles/r03s3_stft64k_tone_precision.txt: the same at every scale, with or without the
    noise floor): the max error is judged against the peak here, the L2 error against the norm
    (SURVEY 8c's two measures, the first one normalised where it is well posed).  A NaN
    sample turns exactly the frames that contain it into NaN (the butterflies spread it over
    every bin) and leaves the others finite."""
    from sdrgpu.device import DeviceBuffer
    n, hop, nfr = 65536, 32768, 12
    total = hop * nfr
    rng = np.random.default_rng(64)
    t = np.arange(total)
    base = (np.exp(2j * np.pi * 0.1234567 * t) + 1e-6 * cplx(rng, total)).astype(np.complex64)
    base[4 * hop:6 * hop] = 0          # frames 4 and 5 partly, frame 5 wholly (span 4..5) zero
    for scale in (1e-30, 1.0, 1e30):
        x = (base * np.float32(scale)).astype(np.complex64)
        s = sdr.fft.Stft(n, hop)
        dx = DeviceBuffer.from_numpy(x)
        dy = DeviceBuffer.empty(nfr * n)
        assert s.process_dev(dx.ptr, total, dy.ptr, nfr) == nfr
        s.sync()
        y = dy.download(nfr * n).reshape(nfr, n)
        assert np.isfinite(y).all(), scale
        assert not y[5].any(), "all-zero frame"
        for j in (0, 3, 4, 6, nfr - 1):
            span = _c3_frame_span(x, j, n, hop).astype(np.complex128)
            ref = np.fft.fftshift(np.fft.fft(span)) / np.sqrt(n)
            d = np.abs(y[j].astype(np.complex128) - ref)
            peak = np.abs(ref).max()
            assert d.max() <= 1e-5 * peak, (scale, j, d.max() / peak)
            assert np.linalg.norm(d) <= 1e-5 * np.linalg.norm(ref), (scale, j)
    x = base.copy()
    x[7 * hop + 123] = np.nan          # inside frames 7 and 8 (spans [6h, 8h) and [7h, 9h))
    s = sdr.fft.Stft(n, hop)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nfr * n)
    assert s.process_dev(dx.ptr, total, dy.ptr, nfr) == nfr
    s.sync()
    y = dy.download(nfr * n).reshape(nfr, n)
    for j in range(nfr):
        if j in (7, 8):
            assert np.isnan(y[j]).all(), f"frame {j} holds the NaN"
        else:
            assert np.isfinite(y[j]).all(), f"frame {j} does not"


def _check_db(y_db, ref_c, what):
    """dB output vs the oracle's complex bins: the magnitudes 10^(dB/20) within the FIR/FFT
    parity bound (1e-5 of RMS), and 20 log10 |X| (src/plot/complexseries.rs:90-92)
    within 1e-4 dB on bins no more than 20 dB below the frame's RMS."""
    mag = np.abs(ref_c.astype(np.complex128))
    assert_parity(10.0 ** (y_db.astype(np.float64) / 20.0), mag, what=what)
    ref_db = 20.0 * np.log10(mag)
    keep = mag > 0.1 * np.sqrt(np.mean(mag ** 2))
    assert np.abs(y_db[keep] - ref_db[keep]).max() < 1e-4, what


@pytest.mark.parametrize("n", [1024, 1000, 65536, 14400])
def test_fft_db_output(sdr, oracle, n):
    """The fused |X| -> dB store (one f32 per bin)."""
    rng = np.random.default_rng(n)
    x = cplx(rng, 2 * n).reshape(2, n)
    y = sdr.fft.FftPlan(n, output="db").exec(x)
    assert y.dtype == np.float32 and y.shape == (2, n)
    for c in range(2):
        ref = oracle.fft_frame(x[c]) if n <= 20000 else \
            np.fft.fftshift(np.fft.fft(x[c].astype(np.complex128))) / np.sqrt(n)
        _check_db(y[c], ref, f"db n={n} frame {c}")
    r = sdr.fft.FftPlan(n, output="db").exec_real(x.real.astype(np.float32))
    full = np.fft.fftshift(np.fft.fft(x.real.astype(np.float64), axis=1), axes=1) / np.sqrt(n)
    assert r.shape == full[:, n // 2:].shape
    for c in range(2):
        _check_db(r[c], full[c, n // 2:], f"rfft db n={n} frame {c}")


def test_stft_db_output(sdr, oracle):
    rng = np.random.default_rng(5)
    n, hop = 65536, 32768
    x = cplx(rng, hop * 5 + 11)
    y = sdr.fft.Stft(n, hop, output="db").process(x)
    ref = oracle.stft(x, n, hop, nthreads=8)
    assert y.shape == ref.shape and y.dtype == np.float32
    for j in range(ref.shape[0]):
        _check_db(y[j], ref[j], f"stft db frame {j}")


def test_stft_u8_input(sdr, oracle):
    from sdrgpu import _lib
    rng = np.random.default_rng(6)
    # (1000, 500): examples/live.rs's rtl.listen().window(..).decimate(..) on the compile-time
    # 1000-point plan; 14400: the other compile-time plan
    for n, hop in ((4096, 1000), (65536, 32768), (1000, 500), (14400, 7200)):
        iq = rng.integers(0, 256, 2 * (hop * 4 + 5), dtype=np.uint8)
        s = sdr.fft.Stft(n, hop, input_kind=_lib.CU8)
        y = np.concatenate([s.process(iq[:2 * 777]), s.process(iq[2 * 777:])])
        ref = oracle.stft(oracle.u8_to_c64(iq), n, hop, nthreads=8)
        assert y.shape == ref.shape
        for j in range(ref.shape[0]):
            assert_parity(y[j], ref[j], what=f"u8 stft n={n} frame {j}")


@pytest.mark.parametrize("n,hop", [(1000, 500), (1000, 1300), (1024, 512), (4096, 1000), (1200, 600),
                                   (6000, 3000), (14400, 7200)])
@pytest.mark.parametrize("u8", [False, True])
def test_stft_full_workgroup_gather(sdr, oracle, n, hop, u8):
    """Streams long enough that most workgroups take the full-workgroup 32-bit gather / store
    (fft_frames.hpp gather_tile_ct / gather_tile fast path), the first ones the history path and
    the last a ragged tile, in two blocks (the second starting from carried history); c64 and
    dB outputs against the oracle.  Compile-time plans (1000, 14400), power-of-two tiles (1024,
    4096), the generic mixed-radix tile (1200, 6000)."""
    from sdrgpu import _lib
    rng = np.random.default_rng(n + hop + u8)
    n_in = hop * 37 + 123
    if u8:
        iq = rng.integers(0, 256, 2 * n_in, dtype=np.uint8)
        x, cut, kind = oracle.u8_to_c64(iq), 2 * (hop * 9 + 17), _lib.CU8
        parts = (iq[:cut], iq[cut:])
    else:
        x = cplx(rng, n_in)
        cut, kind = hop * 9 + 17, _lib.C64
        parts = (x[:cut], x[cut:])
    ref = oracle.stft(x, n, hop, nthreads=8)
    s = sdr.fft.Stft(n, hop, input_kind=kind)
    y = np.concatenate([s.process(p) for p in parts])
    assert y.shape == ref.shape
    for j in range(ref.shape[0]):
        assert_parity(y[j], ref[j], what=f"stft n={n} hop={hop} u8={u8} frame {j}")
    s = sdr.fft.Stft(n, hop, input_kind=kind, output="db")
    yd = np.concatenate([s.process(p) for p in parts])
    assert yd.shape == ref.shape and yd.dtype == np.float32
    for j in range(0, ref.shape[0], 5):
        _check_db(yd[j], ref[j], f"stft db n={n} hop={hop} u8={u8} frame {j}")
