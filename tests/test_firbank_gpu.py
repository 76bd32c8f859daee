"""GPU parity of the FIR BANK at decimation 1 -- the hot kernel of configs[3] (matched
filter in front of the PLL, 1024 channels) and configs[4] (8192-channel channelizer):
`fir_mxh_kernel<NCH, ..., D=1>` with its grid-spread history carry, plus the overlap-save
path, against the oracle's per-channel Fir (src/filter/fir.rs:23-32 per channel,
src/main.rs:41-49 for the chain).  Tolerance: 1e-5 of RMS per channel;
the PLL downstream of the bank is bit-exact to the oracle PLL fed the same samples."""
import numpy as np
import pytest

from conftest import assert_parity

pytestmark = pytest.mark.gpu


def cplx(rng, shape):
    return (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)


def algo_id(name):
    from sdrgpu import _lib
    return {"auto": _lib.FIR_AUTO, "os": _lib.FIR_OVERLAP_SAVE, "mx": _lib.FIR_MATRIX,
            "direct": _lib.FIR_DIRECT}[name]


def bank(sdr, taps, nch, algo="auto", D=1):
    return sdr.filter.FirBank(taps, nch, sample_kind=1, decim=D, algorithm=algo_id(algo))


def check_channels(y, ref, what):
    assert y.shape == ref.shape, (what, y.shape, ref.shape)
    for c in range(ref.shape[0]):
        assert_parity(y[c], ref[c], what=f"{what} ch{c}")


# (nch, n, K): K = 255 -> fir_mxh_kernel<9,...,1>; K = 127 -> <5,...,1>
SHAPES = [(2, 20000, 255), (37, 5000, 255), (1024, 3000, 255), (64, 4096, 127),
          (3, 777, 255)]


@pytest.mark.parametrize("algo", ["auto", "os"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "nch{}n{}K{}".format(*s))
def test_firbank_d1_parity(sdr, oracle, shape, algo):
    """Ragged even blocks (the MFMA path needs an even channel stride) carry state."""
    from sdrgpu import _lib
    nch, n, K = shape
    rng = np.random.default_rng(nch * 7 + K)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = cplx(rng, (nch, n))
    ref = oracle.fir_batch(taps, x, 1, nthreads=16)
    b = bank(sdr, taps, nch, algo)
    cuts = sorted({min(c, n) for c in (0, 2, 258, 258 + 1024, n // 2 * 2, n)})
    parts = []
    for a, e in zip(cuts[:-1], cuts[1:]):
        if e <= a:
            continue
        parts.append(b.process(x[:, a:e]))
        if algo == "auto" and (e - a) % 2 == 0:
            assert b.last_algorithm() == _lib.FIR_MATRIX, (a, e)
        if algo == "os":
            assert b.last_algorithm() == _lib.FIR_OVERLAP_SAVE
    check_channels(np.concatenate(parts, axis=1), ref, f"D1 {algo} {shape}")


def test_firbank_d1_odd_blocks_fall_back(sdr, oracle):
    """Odd block lengths give an odd device stride on the host path: another kernel runs
    that block and the stream state stays consistent with the MFMA blocks around it."""
    from sdrgpu import _lib
    rng = np.random.default_rng(31)
    nch, K = 9, 255
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = cplx(rng, (nch, 6001))
    ref = oracle.fir_batch(taps, x, 1)
    b = bank(sdr, taps, nch)
    y0 = b.process(x[:, :2000])
    assert b.last_algorithm() == _lib.FIR_MATRIX
    y1 = b.process(x[:, 2000:3001])             # odd: not the MFMA kernel
    assert b.last_algorithm() != _lib.FIR_MATRIX
    y2 = b.process(x[:, 3001:])
    assert b.last_algorithm() == _lib.FIR_MATRIX
    check_channels(np.concatenate([y0, y1, y2], axis=1), ref, "odd fallback")


@pytest.mark.parametrize("ld_pad", [0, 1, 2, 7])
def test_firbank_d1_device_leading_dims(sdr, oracle, ld_pad):
    """process_dev with padded (odd and even) input / output leading dimensions."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(40 + ld_pad)
    nch, n, K = 33, 4100, 255
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = cplx(rng, (nch, n))
    ld_in, ld_out = n + ld_pad, n + 3 + ld_pad
    xp = np.zeros((nch, ld_in), np.complex64)
    xp[:, :n] = x
    b = bank(sdr, taps, nch)
    dx = DeviceBuffer.from_numpy(xp)
    dy = DeviceBuffer.empty(nch * ld_out, np.complex64)
    dy.fill_zero()
    half = 2048
    assert b.process_dev(dx.ptr, ld_in, half, dy.ptr, ld_out) == half
    if ld_in % 2 == 0:
        assert b.last_algorithm() == _lib.FIR_MATRIX
    assert b.process_dev(dx.ptr + 8 * half, ld_in, n - half, dy.ptr + 8 * half, ld_out) == n - half
    b.sync()
    y = dy.download().reshape(nch, ld_out)
    assert np.all(y[:, n:] == 0), "wrote past n_out inside the leading dimension"
    check_channels(y[:, :n], oracle.fir_batch(taps, x, 1), f"ld_pad {ld_pad}")


def test_firbank_d1_reset_and_clone(sdr, oracle):
    rng = np.random.default_rng(43)
    nch, n, K = 16, 8192, 255
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = cplx(rng, (nch, n))
    b = bank(sdr, taps, nch)
    a = b.process(x[:, :3000])
    c = b.clone()                 # #[derive(Clone)] snapshot (fir.rs:6)
    b1 = b.process(x[:, 3000:])
    b2 = c.process(x[:, 3000:])
    assert np.array_equal(b1, b2)
    b.reset()
    assert np.array_equal(b.process(x[:, :3000]), a)
    check_channels(np.concatenate([a, b1], axis=1), oracle.fir_batch(taps, x, 1), "clone")


def test_firbank_d1_channelizer_full_width(sdr, oracle):
    """configs[4]'s channel count (8192 x 255 taps, D = 1) at 2^12 samples per channel,
    in two blocks through device buffers (the bench's resident layout)."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    import scipy.signal as ss
    rng = np.random.default_rng(44)
    nch, n = 8192, 4096
    taps = ss.firwin(255, 0.2).astype(np.float32)
    x = (cplx(rng, (nch, n)) * np.float32(0.3))
    b = bank(sdr, taps, nch)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nch * n, np.complex64)
    assert b.process_dev(dx.ptr, n, 1536, dy.ptr, n) == 1536
    assert b.last_algorithm() == _lib.FIR_MATRIX
    assert b.process_dev(dx.ptr + 8 * 1536, n, n - 1536, dy.ptr + 8 * 1536, n) == n - 1536
    b.sync()
    y = dy.download().reshape(nch, n)
    ref = oracle.fir_batch(taps, x, 1, nthreads=16)
    mx = np.abs(y.astype(np.complex128) - ref).max(axis=1)
    rms = np.sqrt(np.mean(np.abs(ref.astype(np.complex128)) ** 2, axis=1))
    worst = float((mx / rms).max())
    assert worst <= 1e-5, f"worst channel max/rms {worst:.3e}"
    l2 = np.linalg.norm(y - ref) / np.linalg.norm(ref)
    assert l2 <= 1e-5


@pytest.mark.parametrize("nch,n,cut", [(128, 16384, 6000), (1024, 9000, 3002)],
                         ids=["nch128", "nch1024_configs3"])
def test_c4_matched_filter_into_pll_chain(sdr, oracle, nch, n, cut):
    """configs[3]: matched-filter bank (D = 1, MFMA) -> batched PLL (src/main.rs:41-49) on
    device buffers, at 128 channels and at configs[3]'s stated width of 1024 channels
    (16 PLL workgroups, n >= 8192 in two ragged even blocks).  The bank is checked against
    the oracle's Fir within 1e-5; the PLL outputs and lock flags are bit-exact to the oracle
    PLL (src/filter/pll.rs:70-85) fed the same (downloaded) bank output."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    import scipy.signal as ss
    from test_pll_gpu import RATE, fm_channels, main_rs_design, oracle_params
    rng = np.random.default_rng(45 + nch)
    x = fm_channels(rng, nch, n)
    taps = ss.firwin(255, 0.2).astype(np.float32)
    b = bank(sdr, taps, nch)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nch * n, np.complex64)
    do = DeviceBuffer.empty(nch * n, np.float32)
    dl = DeviceBuffer.empty(nch * n, np.uint8)
    for a, e in ((0, cut), (cut, n)):
        assert b.process_dev(dx.ptr + 8 * a, n, e - a, dy.ptr + 8 * a, n) == e - a
        assert b.last_algorithm() == _lib.FIR_MATRIX
        b.sync()
        pll.process_dev(dy.ptr + 8 * a, n, e - a, do.ptr + 4 * a, dl.ptr + a, n)
    pll.sync()
    y = dy.download().reshape(nch, n)
    check_channels(y, oracle.fir_batch(taps, x, 1, nthreads=16), "matched filter")
    out = do.download(dtype=np.float32).reshape(nch, n)
    lk = dl.download(dtype=np.uint8).reshape(nch, n)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), y, nthreads=16)
    assert np.array_equal(lk, ref_lk), f"lock mask differs in {np.sum(lk != ref_lk)} samples"
    assert np.array_equal(out, ref_out), f"{np.sum(out != ref_out)} PLL outputs differ"
    assert lk.any() and out[lk.astype(bool)].std() > 0  # the chain locks and demodulates


@pytest.mark.parametrize("K,n", [(127, 4096), (255, 4096), (127, 1 << 15), (255, 1 << 15)])
def test_pll_beside_concurrent_mfma_bank(sdr, oracle, K, n):
    """The main.rs PLL (src/main.rs:41-46; src/filter/pll.rs:70-85) over 1024 channels while
    matched-filter bank launches (D = 1 MFMA kernel, src/filter/fir.rs:23-32 per channel) stream
    over other buffers on another stream for the PLL's whole run.  n = 4096 runs the serial split
    kernel; n = 2^15 is 8 segments of 4 Ki per channel, so the automatic plan runs the
    time-parallel pll_seg / pll_refix / pll_fix kernels (configs[3]'s default) beside the bank.
    Outputs and lock flags array_equal to the oracle PLL; the bank's last block within tolerance.
    This is a concurrency smoke test, not the guard for the co-residency fault of DESIGN.md 3.6:
    the shipped banks and PLL kernels cannot share a SIMD (both claim its register file), so it
    cannot reproduce that fault; tests/test_kernel_resources_cpu.py checks the claims."""
    from sdrgpu.device import DeviceBuffer
    import scipy.signal as ss
    from test_pll_gpu import RATE, fm_channels, main_rs_design, oracle_params
    rng = np.random.default_rng(500 + K + n)
    nch = 1024
    x = fm_channels(rng, nch, n)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    tp = n >= 1 << 15
    assert (pll.time_parallel_plan(n)[0] > 0) == tp
    dx = DeviceBuffer.from_numpy(x)
    do = DeviceBuffer.empty(nch * n, np.float32)
    dl = DeviceBuffer.empty(nch * n, np.uint8)
    taps = ss.firwin(K, 0.2).astype(np.float32)
    nb_ch, nb = 1024, 16384
    xb = cplx(rng, (nb_ch, nb)) * np.float32(0.3)
    b = bank(sdr, taps, nb_ch)
    dxb = DeviceBuffer.from_numpy(xb)
    dyb = DeviceBuffer.empty(nb_ch * nb, np.complex64)
    b.sync()
    pll.process_dev(dx.ptr, n, n, do.ptr, dl.ptr, n)      # the PLL on its stream ...
    reps = 24                                              # ... beside ~24 bank launches
    for _ in range(reps):
        assert b.process_dev(dxb.ptr, nb, nb, dyb.ptr, nb) == nb
    b.sync()
    pll.sync()
    if tp:
        assert pll.last_time_parallel()[0] == n // 4096  # segments per channel
    out = do.download(dtype=np.float32).reshape(nch, n)
    lk = dl.download(dtype=np.uint8).reshape(nch, n)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), x, nthreads=16)
    bad = (out != ref_out) | (lk != ref_lk)
    if bad.any():
        chs = np.unique(np.nonzero(bad)[0])
        raise AssertionError(f"PLL beside the bank: {int(bad.sum())} samples wrong in {chs.size} "
                             f"channels (lanes {sorted(set((chs % 64).tolist()))[:16]})")
    assert lk.any() and out[lk.astype(bool)].std() > 0
    # the bank's last launch: the stream of reps identical blocks, checked on a few channels
    y = dyb.download().reshape(nb_ch, nb)
    for c in (0, 517, nb_ch - 1):
        stream = np.tile(xb[c], reps)
        ref = oracle.Fir(taps, 1, sample_kind=1).process(stream)[-nb:]
        assert_parity(y[c], ref, what=f"bank ch {c}")
