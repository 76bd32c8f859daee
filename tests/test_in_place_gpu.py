"""GPU tests: device-pointer calls whose output range overlaps their input range.

The reference's blocks take an input slice and return a fresh Vec (Fir::apply,
src/filter/fir.rs:23-32; fft::fft, src/fft.rs:3-28), so aliasing has no reference behaviour to
mirror; the C ABI defines it as "same results as out of place" (include/sdrgpu.h).  The FIR, FFT
and STFT kernels store output tiles while other workgroups still read the input under them, so
the handles copy an overlapped input first (unalias_input, abi_common.hpp).  Each case runs the
same blocks out of place on one handle and in place on another and requires identical bits, plus
parity with the oracle on the FIR."""
import numpy as np
import pytest

from conftest import assert_parity

pytestmark = pytest.mark.gpu


def cplx(rng, n):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)


def _fir(sdr, taps, sk, D, algo):
    from sdrgpu import _lib
    a = {"auto": _lib.FIR_AUTO, "direct": _lib.FIR_DIRECT, "os": _lib.FIR_OVERLAP_SAVE,
         "mx": _lib.FIR_MATRIX}[algo]
    return sdr.filter.Fir(taps, decim=D, sample_kind=sk, algorithm=a).design(2.4e6)


FIR_CASES = [
    # (sample kind, ntaps, decim, algorithm, output offset in bytes from the input pointer)
    (1, 255, 4, "mx", 0),          # configs[1] shape, d_out == d_in
    (1, 255, 4, "mx", 4096 * 8),   # output starts inside the input, past the first tiles
    (1, 255, 4, "os", 0),
    (1, 255, 4, "direct", 0),
    (1, 255, 1, "auto", 0),
    (2, 255, 4, "mx", 0),          # rtl_tcp u8: 2-byte inputs under 8-byte outputs
    (0, 127, 1, "auto", 0),        # configs[0] shape (f32)
]


@pytest.mark.parametrize("sk,K,D,algo,off", FIR_CASES)
def test_fir_in_place_matches_out_of_place(sdr, oracle, sk, K, D, algo, off):
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(500 + K + D + sk)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    n = 1 << 18
    if sk == 2:
        x = rng.integers(0, 256, 2 * n, dtype=np.uint8)
        ref_in = oracle.u8_to_c64(x)
    elif sk == 1:
        x = ref_in = cplx(rng, n)
    else:
        x = ref_in = rng.standard_normal(n).astype(np.float32)
    oelem = 4 if sk == 0 else 8
    fa, fb = _fir(sdr, taps, sk, D, algo), _fir(sdr, taps, sk, D, algo)
    half = n // 2
    ib = x.nbytes // 2                       # bytes of one half block
    ys_a, ys_b = [], []
    for h in range(2):
        blk = np.ascontiguousarray(x[h * (x.size // 2):(h + 1) * (x.size // 2)])
        n_out = fa.output_len(half)
        dx = DeviceBuffer.from_numpy(blk)
        dy = DeviceBuffer.empty(n_out * oelem, np.uint8)
        assert fa.process_dev(dx.ptr, half, dy.ptr, n_out) == n_out
        fa.sync()
        ys_a.append(dy.download(n_out * oelem, np.uint8))
        # in place: one buffer holds the input at 0 and the output at `off`
        db = DeviceBuffer(max(ib, off + n_out * oelem) + 256)
        db.upload(blk)
        assert fb.process_dev(db.ptr, half, db.ptr + off, n_out) == n_out
        fb.sync()
        ys_b.append(db.download(n_out * oelem, np.uint8, offset_bytes=off))
        assert fb.last_algorithm() == fa.last_algorithm()
        assert fb.last_kernel() == fa.last_kernel()
    a, b = np.concatenate(ys_a), np.concatenate(ys_b)
    assert np.array_equal(a, b), f"in place differs from out of place ({algo}, off {off})"
    odt = np.float32 if sk == 0 else np.complex64
    ref = oracle.Fir(taps, D, sample_kind=0 if sk == 0 else 1).process(ref_in)
    assert_parity(b.view(odt), ref, what=f"in place {algo} sk{sk} D{D}")


def test_firbank_in_place_matches_out_of_place(sdr):
    """The D = 1 MFMA bank (64 channels) with each output row written over its input row."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(520)
    K, nch, n = 255, 64, 1 << 14
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    x = cplx(rng, nch * n).reshape(nch, n)
    ba = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1)
    bb = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(nch * n)
    assert ba.process_dev(dx.ptr, n, n, dy.ptr, n) == n
    ba.sync()
    assert bb.process_dev(dx.ptr, n, n, dx.ptr, n) == n
    bb.sync()
    assert bb.last_kernel() == ba.last_kernel()
    assert np.array_equal(dx.download(), dy.download())


@pytest.mark.parametrize("n,count", [(1024, 64), (14400, 9), (4099, 17), (1 << 16, 4)])
def test_fft_in_place_matches_out_of_place(sdr, n, count):
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(n)
    x = cplx(rng, n * count)
    p = sdr.fft.FftPlan(n)
    dx, dy = DeviceBuffer.from_numpy(x), DeviceBuffer.empty(n * count)
    p.exec_dev(dx.ptr, dy.ptr, count)
    p.exec_dev(dx.ptr, dx.ptr, count)
    p.sync()
    assert np.array_equal(dx.download(), dy.download())
    # rfft: the half spectra written over the front of the real frames
    xr = rng.standard_normal(n * count).astype(np.float32)
    nb = count * (n - n // 2)
    dr = DeviceBuffer(max(xr.nbytes, nb * 8))
    dr.upload(xr)
    do = DeviceBuffer.empty(nb)
    p.exec_real_dev(dr.ptr, do.ptr, count)
    p.exec_real_dev(dr.ptr, dr.ptr, count)
    p.sync()
    assert np.array_equal(dr.download(nb, np.complex64), do.download())


def test_stft_in_place_matches_out_of_place(sdr):
    """Frames written over the samples they are cut from, over two streamed blocks (the carry
    kernel re-reads the block's tail after the frames are stored)."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(530)
    n, hop, blk = 4096, 1000, 20000
    x = cplx(rng, 2 * blk)
    sa, sb = sdr.fft.Stft(n, hop), sdr.fft.Stft(n, hop)
    for h in range(2):
        part = x[h * blk:(h + 1) * blk]
        nf = sa.output_len(blk)
        assert nf > 0
        dx, dy = DeviceBuffer.from_numpy(part), DeviceBuffer.empty(nf * n)
        assert sa.process_dev(dx.ptr, blk, dy.ptr, nf) == nf
        db = DeviceBuffer(max(part.nbytes, nf * n * 8))
        db.upload(part)
        assert sb.process_dev(db.ptr, blk, db.ptr, nf) == nf
        sa.sync()
        sb.sync()
        assert np.array_equal(db.download(nf * n, np.complex64), dy.download()), f"block {h}"
