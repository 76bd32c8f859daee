"""GPU parity tests: sdrgpu FIR / FIR-decimate / FIR bank (via the C ABI) vs the oracle.

Reference semantics: Fir::apply (src/filter/fir.rs:23-32) + Decimate
(src/signal/adapters/mod.rs:30-37).  Tolerance: 1e-5 of RMS.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, assert_parity, rms_rel_err

pytestmark = pytest.mark.gpu

GOLD = os.path.join(ROOT, "tests", "golden")


def cplx(rng, n, dtype=np.complex64):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(dtype)


def make_case(rng, sk, tk, K, n):
    taps = rng.standard_normal(K).astype(np.float32) / np.sqrt(K)
    if tk == 1:
        taps = (taps + 1j * rng.standard_normal(K) / np.sqrt(K)).astype(np.complex64)
    x = cplx(rng, n) if sk == 1 else rng.standard_normal(n).astype(np.float32)
    return taps, x


ALGOS = ["direct", "os", "mx", "auto"]


def fir(sdr, taps, sk, D, algo="auto"):
    from sdrgpu import _lib
    a = {"auto": _lib.FIR_AUTO, "direct": _lib.FIR_DIRECT, "os": _lib.FIR_OVERLAP_SAVE,
         "mx": _lib.FIR_MATRIX}[algo]
    try:
        return sdr.filter.Fir(taps, decim=D, sample_kind=sk, algorithm=a).design(2.4e6)
    except _lib.SdrGpuError as e:
        if e.code == _lib.ERR_UNSUPPORTED and algo in ("os", "mx"):
            pytest.skip(f"{algo} does not cover this shape")
        raise


CASES = [
    # (sample_kind, tap_kind, ntaps, decim, n)
    (1, 0, 255, 4, 10000),     # configs[1] shape
    (0, 0, 127, 1, 5000),      # configs[0] shape
    (1, 1, 63, 3, 3001),       # complex taps
    (1, 0, 1, 1, 100),         # single tap (no history)
    (1, 0, 5, 7, 33),          # D > K
    (0, 0, 300, 2, 2000),
    (1, 0, 255, 1, 70000),     # many workgroups
    (1, 0, 255, 4, 1 << 18),
    (1, 0, 2000, 16, 40000),   # long filter, heavy decimation
    (1, 0, 33, 64, 50000),     # LDS fallback path (very large D)
    (1, 1, 255, 4, 20000),
    (0, 0, 64, 8, 9999),
    (1, 0, 255, 2, 30000),     # overlap-save D=2
    (1, 0, 255, 8, 30000),     # overlap-save D=8
    (1, 1, 1000, 1, 20000),    # overlap-save D=1, long complex filter
    (1, 0, 2, 4, 5000),        # shortest filter with history
    (1, 0, 255, 4, 333333),    # MFMA path: many segments, ragged last segment
    (1, 0, 61, 4, 7777),       # MFMA path: short filter (4 chunks)
    (1, 0, 100, 2, 20001),     # MFMA D=2, odd length
    (1, 0, 200, 8, 65537),     # MFMA D=8
    (1, 0, 1, 2, 1000),        # MFMA single tap
]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("case", CASES, ids=lambda c: "sk{}tk{}K{}D{}n{}".format(*c))
def test_fir_parity(sdr, oracle, case, algo):
    sk, tk, K, D, n = case
    rng = np.random.default_rng(hash(case) % 2**32)
    taps, x = make_case(rng, sk, tk, K, n)
    ref = oracle.Fir(taps, D, sample_kind=sk).process(x)
    y = fir(sdr, taps, sk, D, algo).process(x)
    assert y.shape == ref.shape
    assert_parity(y, ref, what=str(case))


@pytest.mark.parametrize("scale", [1e-30, 1e-6, 1e6, 1e30])
def test_fir_mx_dynamic_range(sdr, oracle, scale):
    """The exact 3-way bf16 split keeps f32's exponent range: tiny and huge inputs."""
    rng = np.random.default_rng(17)
    taps, x = make_case(rng, 1, 0, 255, 20000)
    x = (x * np.float32(scale)).astype(np.complex64)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(x)
    y = fir(sdr, taps, 1, 4, "mx").process(x)
    assert_parity(y, ref, what=f"scale {scale}")


@pytest.mark.parametrize("phase", [0, 1, 2, 3])
def test_fir_mx_decimation_phase(sdr, oracle, phase):
    """Every decimation phase (window alignment delta = 0/1) after a ragged first block."""
    rng = np.random.default_rng(23 + phase)
    taps, x = make_case(rng, 1, 0, 255, 30000)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(x)
    f = fir(sdr, taps, 1, 4, "mx")
    y = np.concatenate([f.process(x[:phase + 1]), f.process(x[phase + 1:])])
    assert_parity(y, ref, what=f"phase {phase}")


def test_fir_mx_unaligned_device_pointer(sdr, oracle):
    """An input pointer that is not 16-byte aligned falls back to another path."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(29)
    taps, x = make_case(rng, 1, 0, 255, 40001)
    f = fir(sdr, taps, 1, 4, "mx")
    dx = DeviceBuffer.from_numpy(x)
    n = x.size - 1
    n_out = f.output_len(n)
    dy = DeviceBuffer.empty(n_out, np.complex64)
    assert f.process_dev(dx.ptr + 8, n, dy.ptr, n_out) == n_out
    f.sync()
    assert_parity(dy.download(), oracle.Fir(taps, 4, sample_kind=1).process(x[1:]))


@pytest.mark.parametrize("name", ["fir_c1.npz", "fir_c2.npz", "fir_cc.npz"])
def test_fir_golden(sdr, name):
    g = np.load(os.path.join(GOLD, name), allow_pickle=False)
    sk = int(np.iscomplexobj(g["x"]))
    y = fir(sdr, g["taps"], sk, int(g["decim"])).process(g["x"])
    assert_parity(y, g["y"], what=name)


@pytest.mark.parametrize("algo", ALGOS)
def test_fir_block_partition_invariance(sdr, oracle, algo):
    rng = np.random.default_rng(7)
    taps, x = make_case(rng, 1, 0, 255, 50000)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(x)
    whole = fir(sdr, taps, 1, 4, algo).process(x)
    f = fir(sdr, taps, 1, 4, algo)
    parts, i = [], 0
    for step in (1, 2, 3, 5, 100, 253, 254, 255, 256, 4095, 1, 7777, 13, 20000):
        parts.append(f.process(x[i:i + step]))
        i += step
    parts.append(f.process(x[i:]))
    y = np.concatenate(parts)
    assert_parity(y, ref, what="chunked")
    if algo == "direct":
        assert np.array_equal(y, whole)  # same per-output arithmetic, any partition


def test_fir_empty_and_tiny_blocks(sdr, oracle):
    rng = np.random.default_rng(3)
    taps, x = make_case(rng, 1, 0, 255, 20)
    f = fir(sdr, taps, 1, 4)
    assert f.process(x[:0]).size == 0
    o = oracle.Fir(taps, 4, sample_kind=1)
    ys, rs = [], []
    for i in range(20):  # one sample at a time, like Filter::apply
        ys.append(f.process(x[i:i + 1]))
        rs.append(o.process(x[i:i + 1]))
        assert ys[-1].size == rs[-1].size
    assert_parity(np.concatenate(ys), np.concatenate(rs))


def test_fir_apply_single_sample_api(sdr, oracle):
    taps = np.array([0.5, 0.25, 0.125], np.float32)
    f = sdr.filter.Fir(taps, sample_kind=0).design(1.0)
    o = oracle.Fir(taps, 1, sample_kind=0)
    for v in [1.0, 0.0, 0.0, 2.0, -1.0]:
        assert np.isclose(f.apply(v), o.process(np.array([v], np.float32))[0], atol=1e-7)
    fd = sdr.filter.Fir(taps, decim=2, sample_kind=0).design(1.0)
    assert fd.apply(1.0) is None and fd.apply(0.0) is not None


def test_fir_output_cap_error(sdr):
    import ctypes
    from sdrgpu import _lib
    taps = np.ones(8, np.float32)
    f = fir(sdr, taps, 1, 1)
    x = np.ones(100, np.complex64)
    out = np.empty(10, np.complex64)
    got = ctypes.c_size_t()
    rc = _lib.lib().sdrgpu_fir_process(f._h, x.ctypes.data, 100, out.ctypes.data, 10,
                                       ctypes.byref(got))
    assert rc == _lib.ERR_OUTPUT_CAP and got.value == 100
    # a rejected call leaves the state untouched
    ref = np.convolve(x, taps)[:100]
    assert_parity(f.process(x), ref)


def test_fir_reset_and_clone(sdr, oracle):
    rng = np.random.default_rng(11)
    taps, x = make_case(rng, 1, 0, 255, 30000)
    f = fir(sdr, taps, 1, 4)
    a = f.process(x[:12345])
    c = f.clone()  # #[derive(Clone)] snapshot of state (fir.rs:6)
    b1 = f.process(x[12345:])
    b2 = c.process(x[12345:])
    assert np.array_equal(b1, b2)
    f.reset()
    assert np.array_equal(f.process(x[:12345]), a)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(x)
    assert_parity(np.concatenate([a, b1]), ref)


@pytest.mark.parametrize("algo", ["auto", "mx", "os", "direct"])
def test_firbank_parity(sdr, oracle, algo):
    from sdrgpu import _lib
    rng = np.random.default_rng(5)
    nch, n, K, D = 37, 5000, 255, 4
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = cplx(rng, nch * n).reshape(nch, n)
    ref = oracle.fir_batch(taps, x, D, nthreads=8)
    a = {"auto": _lib.FIR_AUTO, "direct": _lib.FIR_DIRECT, "os": _lib.FIR_OVERLAP_SAVE,
         "mx": _lib.FIR_MATRIX}[algo]
    bank = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=D, algorithm=a)
    # 1111 is odd: the MFMA path needs even channel strides and hands that block on
    y = np.concatenate([bank.process(x[:, :1234]), bank.process(x[:, 1234:2345]),
                        bank.process(x[:, 2345:])], axis=1)
    assert y.shape == ref.shape
    for c in range(nch):
        assert_parity(y[c], ref[c], what=f"ch{c}")


def test_fir_device_pointer_path(sdr, oracle):
    """process_dev on device buffers, timed with events on the handle's stream."""
    from sdrgpu.device import DeviceBuffer, Event
    rng = np.random.default_rng(9)
    taps, x = make_case(rng, 1, 0, 255, 1 << 20)
    f = fir(sdr, taps, 1, 4)
    dx = DeviceBuffer.from_numpy(x)
    n_out = f.output_len(x.size)
    dy = DeviceBuffer.empty(n_out, np.complex64)
    e0, e1 = Event(), Event()
    e0.record(f.stream())
    got = f.process_dev(dx.ptr, x.size, dy.ptr, n_out)
    e1.record(f.stream())
    assert got == n_out
    f.sync()
    assert e0.elapsed_ms(e1) > 0
    y = dy.download()
    ref = oracle.Fir(taps, 4, sample_kind=1).process(x)
    assert_parity(y, ref)


def _upload_chunks(buf, n, seed, scale=1.0, chunk=1 << 24):
    for i in range(0, n, chunk):
        r = np.random.default_rng(seed + i // chunk)
        c = ((r.standard_normal(chunk, dtype=np.float32) +
              1j * r.standard_normal(chunk, dtype=np.float32)) * scale).astype(np.complex64)
        buf.upload(c, offset_bytes=8 * i)


@pytest.mark.slow
def test_fir_full_size_c2_properties(sdr, oracle):
    """configs[1] at full size (2^28 c64): spot-check windows against the oracle (the FIR
    is local: output m only depends on inputs g_m-254..g_m) and check linearity."""
    from sdrgpu.device import DeviceBuffer
    import scipy.signal as ss
    n = 1 << 28
    K, D = 255, 4
    taps = ss.firwin(K, 0.2).astype(np.float32)
    dx = DeviceBuffer.empty(n, np.complex64)
    _upload_chunks(dx, n, seed=100)
    f = fir(sdr, taps, 1, D)
    n_out = n // D
    dy = DeviceBuffer.empty(n_out, np.complex64)
    assert f.process_dev(dx.ptr, n, dy.ptr, n_out) == n_out
    f.sync()
    rng = np.random.default_rng(0)
    starts = [0, n_out - 4096] + [int(v) for v in rng.integers(1, n_out - 4096, 6)]
    for m0 in starts:
        g0 = max(0, 4 * m0 - 256)          # covers the 254-sample reach of output m0
        g1 = 4 * (m0 + 4096)
        xin = dx.download(g1 - g0, offset_bytes=8 * g0)
        ref = oracle.Fir(taps, D, sample_kind=1).process(xin)
        skip = m0 - g0 // 4
        ref = ref[skip:skip + 4096]
        y = dy.download(4096, offset_bytes=8 * m0)
        assert_parity(y, ref, what=f"window {m0}")
    # linearity over the whole 2^28 stream: F(2x) == 2 F(x) exactly (power-of-2 scale)
    ys = [dy.download(1 << 20, offset_bytes=8 * m) for m in (0, n_out // 2, n_out - (1 << 20))]
    _upload_chunks(dx, n, seed=100, scale=2.0)
    f2 = fir(sdr, taps, 1, D)
    assert f2.process_dev(dx.ptr, n, dy.ptr, n_out) == n_out
    f2.sync()
    for y1, m in zip(ys, (0, n_out // 2, n_out - (1 << 20))):
        y2 = dy.download(1 << 20, offset_bytes=8 * m)
        assert np.array_equal(y2, 2 * y1)


def mxh_d4_c64_dealing(n_out, cus=256):
    """Host mirror of fir_mxh_launch's c64 D = 4 dealing (fir_mxh.hip:624-637): tiles of 256
    kept outputs, units (runs) of kRunTiles = 2 tiles, unit u dealt grid-strided to wave
    u mod nwaves (a wave walks units w, w + nwaves, ... as one pipeline)."""
    tpc = -(-n_out // 256)
    seg = min(2, tpc)
    units = -(-tpc // seg)
    nwaves = 8 * min(cus, -(-units // 8))
    return {"tiles": tpc, "units": units, "nwaves": nwaves,
            "last_unit_tiles": tpc - (units - 1) * seg,
            "last_tile_outputs": n_out - (tpc - 1) * 256,
            "last_unit_wave": (units - 1) % nwaves,
            "min_units_per_wave": units // nwaves}


def test_fir_mx_run_boundaries_whole_stream(sdr, oracle):
    """The c64 D = 4 kernel deals runs of 2 tiles (512 kept outputs) grid-strided and walks a
    wave's runs as one pipeline: each run's first window re-reads the 256 samples before it
    (fir_mxh.hip:410, :472) and the raw-tile prefetch crosses into the wave's next run.  Two
    device blocks, cut mid-tile (not tile- or run-aligned), carry the history between calls:
      block 1 (1,234,567 outputs): 4823 tiles in 2412 units over 2048 waves -- waves 0-363 own
        two units, and wave 363's second and last unit is ONE partial tile of 135 outputs;
      block 2 (7,154,818 outputs): 27,949 tiles in 13,975 units -- every wave walks >= 6 units
        (6 cross-unit history reloads and prefetches), and the last unit (wave 1686's
        seventh) is again one partial tile (130 outputs).
    (Arithmetic for 256 CUs, checked below through the host mirror of the dealing.)  The
    WHOLE output is compared with the oracle."""
    b1, b2 = mxh_d4_c64_dealing(1234567), mxh_d4_c64_dealing(7154818)
    assert (b1["units"], b1["nwaves"], b1["last_unit_tiles"], b1["last_tile_outputs"],
            b1["last_unit_wave"]) == (2412, 2048, 1, 135, 363)
    assert b2["min_units_per_wave"] >= 6 and b2["last_unit_tiles"] == 1
    assert (b2["last_tile_outputs"], b2["last_unit_wave"]) == (130, 1686)
    from sdrgpu.device import DeviceBuffer
    import scipy.signal as ss
    n = (1 << 25) + 4 * 777 + 3
    K, D = 255, 4
    taps = ss.firwin(K, 0.2).astype(np.float32)
    rng = np.random.default_rng(77)
    x = ((rng.standard_normal(n, dtype=np.float32) + 1j * rng.standard_normal(n, dtype=np.float32))
         * np.float32(0.3)).astype(np.complex64)
    dx = DeviceBuffer.from_numpy(x)
    n_out = n // D
    dy = DeviceBuffer.empty(n_out + 8, np.complex64)
    f = fir(sdr, taps, 1, D)
    cut = 4 * 1234567 + 2
    m1 = f.process_dev(dx.ptr, cut, dy.ptr, n_out + 8)
    m2 = f.process_dev(dx.ptr + 8 * cut, n - cut, dy.ptr + 8 * m1, n_out + 8 - m1)
    f.sync()
    assert (m1, m2) == (1234567, 7154818) and m1 + m2 == n_out
    ref = oracle.fir_batch(taps, x[None, :], D, nthreads=16)[0]
    assert_parity(dy.download(n_out), ref, what="2^25 stream, two blocks")


@pytest.mark.parametrize("algo", ["direct", "mx", "auto"])
def test_time_shard_halo_equivalence(sdr, oracle, algo):
    """Multi-GPU time sharding (bench.py): a shard primed with the 256 preceding samples
    produces exactly the continuation of the unsharded stream."""
    rng = np.random.default_rng(21)
    taps, x = make_case(rng, 1, 0, 255, 80000)
    whole = fir(sdr, taps, 1, 4, algo).process(x)
    half = 40000
    f2 = fir(sdr, taps, 1, 4, algo)
    f2.process(x[half - 256:half])          # halo priming; its outputs belong to shard 0
    y2 = f2.process(x[half:])
    assert y2.shape == whole[half // 4:].shape
    if algo == "direct":
        assert np.array_equal(y2, whole[half // 4:])
    assert_parity(y2, oracle.Fir(taps, 4, sample_kind=1).process(x)[half // 4:])


@pytest.mark.parametrize("weak", [1e-3, 1e-6])
def test_fir_mx_intra_window_dynamic_range(sdr, oracle, weak):
    """A strong burst next to a weak tone inside one staging window of the fp16-split
    kernel (its per-tile scale follows the burst): every 64-output window -- including the
    weak-only ones whose tile shares the burst's scale -- is judged against its OWN RMS."""
    from sdrgpu import _lib
    import scipy.signal as ss
    n, D = 1 << 16, 4
    taps = ss.firwin(255, 0.2).astype(np.float32)
    t = np.arange(n)
    x = (weak * np.exp(2j * np.pi * 0.01 * t)).astype(np.complex64)
    for b0 in range(3000, n, 9000):           # 1.0 bursts, 64 samples long
        x[b0:b0 + 64] += np.exp(2j * np.pi * 0.013 * t[b0:b0 + 64]).astype(np.complex64)
    ref = oracle.Fir(taps, D, sample_kind=1).process(x)
    f = fir(sdr, taps, 1, D, "mx")
    y = f.process(x)
    assert f.last_algorithm() == _lib.FIR_MATRIX
    worst = 0.0
    for w0 in range(0, ref.size - 64, 64):
        mx, _ = rms_rel_err(y[w0:w0 + 64], ref[w0:w0 + 64])
        worst = max(worst, mx)
    assert worst <= 1e-5, f"worst 64-output window max/rms {worst:.3e} (weak {weak})"


@pytest.mark.parametrize("sk,D", [(1, 4), (1, 2), (1, 1), (2, 4), (2, 1)])
def test_fir_mx_silent_stretches(sdr, oracle, sk, D):
    """Exact silence between bursts (c64 zeros; rtl_tcp byte pairs of 128, which convert to 0.0)
    and stretches 60-230 dB apart.  Checked: (1) every output whose 255-sample window is all
    zero is exactly 0.0, as the reference's sequential sum gives; (2) the parity bar (1e-5 of
    the output's RMS); (3) the MFMA kernels' block-floating-point error bound, per
    64-output window w: |y - ref| <= 1e-5 rms_w + 2^-21 max|h| sum_w|x| + 2^-38 M_tile sum|h|.
    The second term is the taps' split / integer rounding (2^-22 of max|h|, fir_mxh.hip hh + hl,
    fir_mxi.hip's three int8 digits); the third is the fp16 sample split under one scale per
    1024-sample tile (fir_mxh.hip): the tile's largest sample M_tile maps to [2^14, 2^15), so a
    sample 2^-29 below it reaches f16's subnormals and one 2^-38 below it flushes to zero.
    A stretch 2^-39 below its neighbour in the same tile (1e-12 next to 0.5 here) is therefore
    not resolved relative to its OWN level, unlike the reference's f32 sum -- measured, and far
    inside (2).  The u8 path has no third term (integer samples)."""
    from sdrgpu import _lib
    import scipy.signal as ss
    rng = np.random.default_rng(600 + 10 * sk + D)
    taps = ss.firwin(255, 0.2).astype(np.float32)
    plan = [("sig", 1.0, 5000), ("zero", 0, 1), ("sig", 1.0, 3000), ("zero", 0, 4096),
            ("sig", 1e-3, 9000), ("zero", 0, 255), ("sig", 0.5, 2000), ("zero", 0, 70000),
            ("sig", 1.0, 7000), ("zero", 0, 1023), ("sig", 1e-2, 30000), ("zero", 0, 3000)]
    if sk == 1:   # c64 also gets a stretch below f16's normal range after silence
        plan[4] = ("sig", 1e-12, 9000)
    n = sum(p[2] for p in plan)
    if sk == 2:
        raw = np.full(2 * n, 128, np.uint8)
        i = 0
        for kind, amp, ln in plan:
            if kind == "sig":
                a = max(1, int(127 * amp))
                raw[2 * i:2 * (i + ln)] = rng.integers(128 - a, 128 + a, 2 * ln).astype(np.uint8)
            i += ln
        x = oracle.u8_to_c64(raw)
        inp = raw
    else:
        x = np.zeros(n, np.complex64)
        i = 0
        for kind, amp, ln in plan:
            if kind == "sig":
                x[i:i + ln] = (amp * (rng.standard_normal(ln) + 1j * rng.standard_normal(ln))).astype(np.complex64)
            i += ln
        inp = x
    ref = oracle.Fir(taps, D, sample_kind=1).process(x)
    f = sdr.filter.Fir(taps, decim=D, sample_kind=sk).design(2.4e6)
    y = f.process(inp)
    assert f.last_kernel() in (_lib.FIR_KERNEL_FP16, _lib.FIR_KERNEL_INT8), f.last_kernel()
    assert y.shape == ref.shape
    g = D - 1 + D * np.arange(ref.size)                   # input index of each kept output
    nz = np.concatenate([[0], np.cumsum(x != 0)])         # nonzero inputs before index i
    silent = nz[g + 1] - nz[np.maximum(g - 254, 0)] == 0
    assert silent.sum() > 1000
    assert np.all(ref[silent] == 0)
    bad = np.nonzero(y[silent] != 0)[0]
    assert bad.size == 0, f"{bad.size} silent outputs nonzero, first at {np.nonzero(silent)[0][bad[0]]}"
    assert_parity(y, ref, what=f"silent stretches sk{sk} D{D}")
    hmax, hsum, ax = float(np.abs(taps).max()), float(np.abs(taps).sum()), np.abs(x)
    worst = (0.0, 0)
    for w0 in range(0, ref.size - 64, 64):
        r = ref[w0:w0 + 64]
        g0, g1 = D - 1 + D * w0, D - 1 + D * (w0 + 63)
        sx = float(ax[max(0, g0 - 254):g1 + 1].sum())
        mt = float(ax[max(0, g0 - 254 - 2048):g1 + 2049].max())
        bound = (1e-5 * np.sqrt(np.mean(np.abs(r) ** 2)) + 2.0 ** -21 * hmax * sx
                 + (2.0 ** -38 * mt * hsum if sk == 1 else 0.0))
        e = float(np.abs(y[w0:w0 + 64] - r).max())
        if e > 0 and e / bound > worst[0]:
            worst = (e / bound, w0)
    print(f"silent sk{sk} D{D}: worst window error {worst[0]:.3f} of the bound (window {worst[1]})")
    assert worst[0] <= 1.0, f"window {worst[1]}: error {worst[0]:.2f} x the bound"


def test_firbank_d1_silent_channels(sdr, oracle):
    """The D = 1 MFMA bank (configs[4]'s kernel) on 8 channels where silence, weak and strong
    stretches fall at different offsets per channel (and two channels are silent throughout):
    all-zero windows give exactly 0.0, every other 64-output window is within 1e-5 of its own
    RMS."""
    from sdrgpu import _lib
    rng = np.random.default_rng(640)
    nch, n, K = 8, 40000, 255
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = np.zeros((nch, n), np.complex64)
    for c in range(2, nch):
        for a0, ln, amp in ((1000 * c, 3000, 1.0), (9000 + 777 * c, 5000, 1e-4), (20000 + 313 * c, 9000, 1e3)):
            x[c, a0:a0 + ln] = (amp * (rng.standard_normal(ln) + 1j * rng.standard_normal(ln))).astype(np.complex64)
    b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1)
    y = b.process(x)
    assert b.last_kernel() == _lib.FIR_KERNEL_FP16
    ref = oracle.fir_batch(taps, x, 1)
    for c in range(nch):
        nz = np.concatenate([[0], np.cumsum(x[c] != 0)])
        g = np.arange(n)
        silent = nz[g + 1] - nz[np.maximum(g - K + 1, 0)] == 0
        assert np.all(ref[c][silent] == 0) and np.all(y[c][silent] == 0), f"ch{c} silent outputs"
        for w0 in range(0, n - 64, 64):
            r = ref[c, w0:w0 + 64]
            if np.any(r):
                mx, _ = rms_rel_err(y[c, w0:w0 + 64], r)
                assert mx <= 1e-5, f"ch{c} window {w0}: max/rms {mx:.3e}"


@pytest.mark.parametrize("K", [1, 129, 130, 255, 257])
def test_fir_mx_decim2_fp16_tiles(sdr, oracle, K):
    """c64 decimate-by-2 on the fp16 x 2 MFMA tiles (fir_mxh.hip at D = 2: 64-byte LDS rows with
    a row swizzle, two 256-output column sets per 1024-sample tile): chunk-count boundary
    K = 129 / 130, ragged blocks (both decimation phases, a partial last tile, carried history),
    then a 3-channel bank."""
    rng = np.random.default_rng(500 + K)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    n = 6 * 1024 + 555
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    ref = oracle.Fir(taps, 2, sample_kind=1).process(x)
    f = sdr.filter.Fir(taps, decim=2, sample_kind=1).design(2.4e6)
    cuts = [0, 3, 1030, 2049, 4100, n]
    y = np.concatenate([f.process(x[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    from sdrgpu import _lib
    assert f.last_algorithm() == _lib.FIR_MATRIX
    assert_parity(y, ref, what=f"K {K}")
    xb = (rng.standard_normal((3, 5000)) + 1j * rng.standard_normal((3, 5000))).astype(np.complex64)
    yb = sdr.filter.FirBank(taps, 3, sample_kind=1, decim=2).process(xb)
    for c in range(3):
        assert_parity(yb[c], oracle.Fir(taps, 2, sample_kind=1).process(xb[c]), what=f"bank K {K} ch {c}")


def _nonfinite_check(y, ref, what):
    """Non-finite outputs exactly where the reference's are (NaN, and inf with its sign); the
    finite ones within the parity bar."""
    assert y.shape == ref.shape, what
    for part in ("real", "imag"):
        a, b = getattr(y, part), getattr(ref, part)
        assert np.array_equal(np.isnan(a), np.isnan(b)), f"{what} {part}: NaN sets differ " \
            f"({np.isnan(a).sum()} vs {np.isnan(b).sum()})"
        assert np.array_equal(np.isposinf(a), np.isposinf(b)) and \
            np.array_equal(np.isneginf(a), np.isneginf(b)), f"{what} {part}: inf sets differ"
    fin = np.isfinite(ref.real) & np.isfinite(ref.imag)
    assert_parity(y[fin], ref[fin], what=what)


NONFINITE = [
    # (samples index, value) groups; each case is one stream of 40000 c64 samples in two blocks
    [(5000, complex(np.nan, 0.0))],
    [(5003, complex(0.0, np.inf))],
    [(0, complex(np.nan, np.nan))],                             # first sample of the stream
    [(10239, complex(-np.inf, 1.0)), (10240, complex(np.inf, 1.0))],  # tile edge, +inf next to -inf
    [(19999, complex(np.nan, 0.0))],                            # last sample of block 1: history
    [(3000, complex(np.inf, 0.0)), (3100, complex(np.nan, 0.0)), (30001, complex(0.0, -np.inf))],
]


@pytest.mark.parametrize("D", [4, 2, 1])
@pytest.mark.parametrize("case", range(len(NONFINITE)))
def test_fir_mx_nonfinite_samples(sdr, oracle, D, case):
    """inf / NaN input samples through the fp16-split MFMA kernel (fir_mxh.hip exact_tile): the
    non-finite outputs are exactly the reference's -- the K outputs whose window holds the
    sample (fir.rs:23-32), NaN where +inf meets -inf -- and every finite output meets the
    parity bar; blocks carry the history (a NaN in block 1's last sample reaches block 2)."""
    from sdrgpu import _lib
    rng = np.random.default_rng(700 + case)
    taps = (rng.standard_normal(255) / np.sqrt(255)).astype(np.float32)
    n = 40000
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    for i, v in NONFINITE[case]:
        x[i] = v
    ref = oracle.Fir(taps, D, sample_kind=1).process(x)
    assert not np.isfinite(ref).all()
    f = sdr.filter.Fir(taps, decim=D, sample_kind=1).design(2.4e6)
    y = np.concatenate([f.process(x[:20000]), f.process(x[20000:])])
    assert f.last_kernel() == _lib.FIR_KERNEL_FP16
    _nonfinite_check(y, ref, f"D{D} case {case}")


def test_firbank_nonfinite_channels(sdr, oracle):
    """The D = 1 MFMA bank with a NaN in one channel and inf in another: nothing leaks across
    channels, and each channel's non-finite outputs are the reference's."""
    from sdrgpu import _lib
    rng = np.random.default_rng(720)
    nch, n = 6, 9000
    taps = (rng.standard_normal(255) / np.sqrt(255)).astype(np.float32)
    x = (rng.standard_normal((nch, n)) + 1j * rng.standard_normal((nch, n))).astype(np.complex64)
    x[1, 4000] = complex(np.nan, 0.0)
    x[4, 1023] = complex(np.inf, -np.inf)
    b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1)
    y = b.process(x)
    assert b.last_kernel() == _lib.FIR_KERNEL_FP16
    ref = oracle.fir_batch(taps, x, 1)
    for c in range(nch):
        _nonfinite_check(y[c], ref[c], f"ch{c}")


NONFINITE_PATHS = [
    # (sample kind, tap kind, ntaps, decim, algorithm, expected kernel)
    (0, 0, 127, 1, "auto", "direct"),      # configs[0]'s shape: the R-blocked direct kernel
    (1, 0, 255, 1, "direct", "direct"),    # fir_direct2 (wave-private, D = 1)
    (1, 0, 255, 4, "direct", "direct"),    # fir_direct4 (D = 4)
    (1, 0, 255, 2, "direct", "direct"),    # fir_direct4 (D = 2)
    (1, 1, 63, 3, "auto", "direct"),       # complex taps, D = 3: the R-blocked direct kernel
    (1, 0, 255, 4, "os", "os"),            # overlap-save, persistent form (D = 4)
    (1, 0, 255, 1, "os", "os"),            # overlap-save, D = 1
    (1, 1, 255, 2, "auto", "os"),          # complex taps: AUTO takes overlap-save
    (1, 0, 255, 8, "auto", "bf16x3"),      # D = 8: the exact bf16 x3 MFMA kernel
    (1, 0, 33, 64, "auto", "direct"),      # very large D: the naive kernel
]


@pytest.mark.parametrize("path", NONFINITE_PATHS, ids=lambda c: "sk{}tk{}K{}D{}{}".format(*c[:5]))
def test_fir_nonfinite_samples_every_path(sdr, oracle, path):
    """inf / NaN samples through every other FIR kernel: padded taps, FFT blocks and the bf16x3
    Toeplitz would carry one beyond the outputs whose window holds it; non-finite outputs are
    replaced by the reference's sum (fir_exact.hpp), so the non-finite sets are the
    reference's and the finite outputs meet the parity bar, over two streamed blocks."""
    from sdrgpu import _lib
    sk, tk, K, D, algo, kern = path
    rng = np.random.default_rng(800 + K + D)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    if tk == 1:
        taps = (taps + 1j * rng.standard_normal(K) / np.sqrt(K)).astype(np.complex64)
    n = 60000
    if sk == 0:
        x = rng.standard_normal(n).astype(np.float32)
        marks = [(100, np.nan), (20000, np.inf), (29999, -np.inf), (45000, np.nan), (45001, np.inf)]
    else:
        x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        marks = [(100, complex(np.nan, 0)), (20000, complex(0, np.inf)), (29999, complex(-np.inf, 1)),
                 (45000, complex(np.nan, np.nan)), (45001, complex(np.inf, -np.inf))]
    for i, v in marks:
        x[i] = v
    ref = oracle.Fir(taps, D, sample_kind=sk).process(x)
    f = fir(sdr, taps, sk, D, algo)
    y = np.concatenate([f.process(x[:30000]), f.process(x[30000:])])
    want = {"direct": _lib.FIR_KERNEL_DIRECT, "os": _lib.FIR_KERNEL_OVERLAP_SAVE,
            "bf16x3": _lib.FIR_KERNEL_BF16X3}[kern]
    assert f.last_kernel() == want, (f.last_kernel(), want)
    if sk == 0:
        assert np.array_equal(np.isnan(y), np.isnan(ref))
        assert np.array_equal(np.isposinf(y), np.isposinf(ref)) and np.array_equal(np.isneginf(y), np.isneginf(ref))
        fin = np.isfinite(ref)
        assert_parity(y[fin], ref[fin], what=str(path))
    else:
        _nonfinite_check(y, ref, str(path))
