"""GPU parity: rtl_tcp u8 IQ ingest fused into the FIR (sample kind CU8) vs the oracle.

Reference chain: RtlTcpConnection::read -> RtlTcpSignal::next, (v - 128) / 128
(src/rtltcp.rs:136-140,156-164), then Signal::filter + Decimate (src/signal/mod.rs:26-48,
src/filter/fir.rs:23-32).  The oracle converts with oracle_u8_to_c64 and filters with its
Fir restatement.  Tolerance 1e-5 of RMS.
"""
import numpy as np
import pytest

from conftest import assert_parity

pytestmark = pytest.mark.gpu


def u8_stream(rng, n):
    return rng.integers(0, 256, size=2 * n, dtype=np.uint8)


CASES = [
    # (ntaps, decim, n, complex_taps)   fused (D=4, f32 taps, K<=257) and converted shapes
    (255, 4, 200000, False),
    (255, 4, 4097, False),
    (61, 4, 30001, False),
    (1, 4, 999, False),
    (127, 1, 20000, False),
    (255, 2, 30000, False),
    (63, 4, 10000, True),
    (300, 4, 20000, False),
]


@pytest.mark.parametrize("algo", ["auto", "mx", "direct"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "K{}D{}n{}c{}".format(*c))
def test_cu8_fir_parity(sdr, oracle, case, algo):
    from sdrgpu import _lib
    K, D, n, ctaps = case
    rng = np.random.default_rng(K * 7 + D + n)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    if ctaps:
        taps = (taps + 1j * rng.standard_normal(K) / np.sqrt(K)).astype(np.complex64)
    raw = u8_stream(rng, n)
    a = {"auto": _lib.FIR_AUTO, "mx": _lib.FIR_MATRIX, "direct": _lib.FIR_DIRECT}[algo]
    try:
        f = sdr.filter.Fir(taps, decim=D, sample_kind=_lib.CU8, algorithm=a).design(2.4e6)
    except _lib.SdrGpuError as e:
        if e.code == _lib.ERR_UNSUPPORTED and algo == "mx":
            pytest.skip("mx does not cover this shape")
        raise
    y = f.process(raw)
    ref = oracle.Fir(taps, D, sample_kind=1).process(oracle.u8_to_c64(raw))
    assert y.dtype == np.complex64 and y.shape == ref.shape
    assert_parity(y, ref, what=str(case))


def test_cu8_block_partition_and_clone(sdr, oracle):
    """State carries across ragged blocks (history kept as converted C64); clone copies it."""
    from sdrgpu import _lib
    rng = np.random.default_rng(5)
    taps = (rng.standard_normal(255) / 16).astype(np.float32)
    raw = u8_stream(rng, 50000)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
    f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    cuts = [0, 3, 1000, 1001, 4096 + 7, 20000, 50000]
    parts = []
    for a, b in zip(cuts[:-2], cuts[1:-1]):
        parts.append(f.process(raw[2 * a:2 * b]))
    g = f.clone()
    tail_f = f.process(raw[2 * cuts[-2]:])
    tail_g = g.process(raw[2 * cuts[-2]:])
    y = np.concatenate(parts + [tail_f])
    assert_parity(y, ref, what="partition")
    np.testing.assert_array_equal(tail_f, tail_g)


def test_cu8_device_path_and_bank(sdr, oracle):
    """Device pointers (fused path, 4-byte aligned) and a channel bank with a leading dim."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(9)
    taps = (rng.standard_normal(255) / 16).astype(np.float32)
    n = 70001
    raw = u8_stream(rng, n)
    f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    dx = DeviceBuffer.from_numpy(raw)
    n_out = f.output_len(n)
    dy = DeviceBuffer.empty(n_out, np.complex64)
    assert f.process_dev(dx.ptr, n, dy.ptr, n_out) == n_out
    f.sync()
    assert_parity(dy.download(), oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw)))
    nch, nb = 5, 9000
    x = rng.integers(0, 256, size=(nch, 2 * nb), dtype=np.uint8)
    bank = sdr.filter.FirBank(taps, nch, sample_kind=_lib.CU8, decim=4)
    y = bank.process(x)
    for c in range(nch):
        ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(x[c]))
        assert_parity(y[c], ref, what=f"bank ch {c}")


def test_cu8_int8_and_fp16_kernels(sdr, oracle):
    """D = 4 u8 blocks take the int8-MFMA kernel (fir_mxi.hip) when the channel bases are
    16-byte aligned and the fp16 kernel (fir_mxh.hip) when they are only 4-byte aligned; both
    meet the tolerance on the same stream, including a bank whose leading dimension breaks the
    16-byte alignment of every other channel (the whole bank then takes the fp16 kernel)."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(31)
    for K in (255, 97):  # 5 and 3 K = 64 chunks
        taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
        n = 3 * 4096 + 1000
        raw = u8_stream(rng, n)
        ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
        for off in (0, 4):  # byte offset of the block: 16-byte aligned, 4-byte aligned
            f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
            dx = DeviceBuffer(2 * n + 16)
            dx.upload(raw, offset_bytes=off)
            n_out = f.output_len(n)
            dy = DeviceBuffer.empty(n_out, np.complex64)
            assert f.process_dev(dx.ptr + off, n, dy.ptr, n_out) == n_out
            f.sync()
            assert f.last_algorithm() == _lib.FIR_MATRIX
            want = _lib.FIR_KERNEL_INT8 if off == 0 else _lib.FIR_KERNEL_FP16
            assert f.last_kernel() == want, (K, off, f.last_kernel())
            assert_parity(dy.download(), ref, what=f"K{K} offset {off}")
    taps = (rng.standard_normal(255) / 16).astype(np.float32)
    for nb in (8192 + 24, 8192 + 26):  # leading dim % 8 == 0 (int8) / != 0 (fp16)
        nch = 4
        x = rng.integers(0, 256, size=(nch, 2 * nb), dtype=np.uint8)
        bank = sdr.filter.FirBank(taps, nch, sample_kind=_lib.CU8, decim=4)
        y = bank.process(x)
        want = _lib.FIR_KERNEL_INT8 if nb % 8 == 0 else _lib.FIR_KERNEL_FP16
        assert bank.last_kernel() == want, (nb, bank.last_kernel())
        for c in range(nch):
            ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(x[c]))
            assert_parity(y[c], ref, what=f"bank nb {nb} ch {c}")


def test_cu8_mixed_kernel_stream(sdr, oracle):
    """One u8 stream whose blocks alternate between 16-byte aligned device buffers (int8
    kernel), 4-byte aligned ones (fp16 kernel) and 2-byte aligned ones (converted to c64 first,
    then the fp16 kernel): the kernel of each block follows the buffer, the history carries
    across the switches, and the whole output stays within the tolerance.  The bits of an
    output depend on which kernel produced it (a documented non-guarantee)."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(404)
    taps = (rng.standard_normal(255) / 16).astype(np.float32)
    n = 9 * 4096 + 1234
    raw = u8_stream(rng, n)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
    f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    cuts = [0, 4096, 8192 + 3, 12289, 20000, 24576, 30001, n]
    offs = [0, 4, 2, 0, 4, 0, 2]
    want = {0: _lib.FIR_KERNEL_INT8, 4: _lib.FIR_KERNEL_FP16,
            2: _lib.FIR_KERNEL_FP16 | _lib.FIR_KERNEL_CU8_CONVERTED}
    dx = DeviceBuffer(2 * n + 32)
    outs = []
    for (a, b), off in zip(zip(cuts[:-1], cuts[1:]), offs):
        dx.upload(raw[2 * a:2 * b], offset_bytes=off)
        m = f.output_len(b - a)
        dy = DeviceBuffer.empty(max(m, 1), np.complex64)
        assert f.process_dev(dx.ptr + off, b - a, dy.ptr, m) == m
        f.sync()
        assert f.last_kernel() == want[off], (a, off, f.last_kernel())
        outs.append(dy.download()[:m])
    assert_parity(np.concatenate(outs), ref, what="mixed-kernel stream")


@pytest.mark.parametrize("scale", [1e-25, 3e-8, 1.0, 5e6, 1e25])
def test_cu8_tap_scale_range(sdr, oracle, scale):
    """The int8 kernel takes the taps as 23-bit integers of h 2^(S): any overall tap scale
    keeps the tolerance (S follows max |h|)."""
    from sdrgpu import _lib
    rng = np.random.default_rng(77)
    taps = (rng.standard_normal(255) / 16 * scale).astype(np.float32)
    raw = u8_stream(rng, 20000)
    f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    y = f.process(raw)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
    assert_parity(y, ref, what=f"tap scale {scale}")


@pytest.mark.parametrize("K", [2, 64, 65, 129, 130, 193, 257, 258])
def test_cu8_int8_tap_count_boundaries(sdr, oracle, K):
    """Tap counts at the int8 kernel's chunk boundaries (3 K = 64 chunks up to K = 129, 5 up to
    257; 258 takes the converting path), over ragged blocks so every decimation phase and a
    partial last tile occur, and the stream history (K - 1 converted samples) is carried."""
    from sdrgpu import _lib
    rng = np.random.default_rng(1000 + K)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    n = 3 * 1024 + 777
    raw = u8_stream(rng, n)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
    f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    cuts = [0, 1, 1030, 1031, 2053, n]
    y = np.concatenate([f.process(raw[2 * a:2 * b]) for a, b in zip(cuts[:-1], cuts[1:])])
    assert_parity(y, ref, what=f"K {K}")


@pytest.mark.parametrize("D,K", [(1, 1), (1, 64), (1, 177), (1, 178), (1, 255), (1, 257),
                                 (2, 1), (2, 161), (2, 162), (2, 255), (2, 257),
                                 (8, 1), (8, 129), (8, 130), (8, 255), (8, 257)])
def test_cu8_int8_no_decimation(sdr, oracle, D, K):
    """D = 1, 2 and 8 u8 blocks on the int8 kernel (D = 1 / 2: 4 / D 256-output column sets per
    1024-sample tile, linear LDS; D = 8: 2048-sample tiles, swizzled LDS): chunk-count
    boundaries (K = 177 / 178 at D = 1, 161 / 162 at D = 2, 129 / 130 at D = 8), ragged blocks
    (every decimation phase), a partial last tile, then a 3-channel bank whose leading
    dimension keeps the 16-byte alignment."""
    from sdrgpu import _lib
    rng = np.random.default_rng(2000 + K + 7 * D)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    n = 5 * 1024 + 333
    raw = u8_stream(rng, n)
    ref = oracle.Fir(taps, D, sample_kind=1).process(oracle.u8_to_c64(raw))
    f = sdr.filter.Fir(taps, decim=D, sample_kind=_lib.CU8).design(2.4e6)
    cuts = [0, 5, 1029, 2048, 4100, n]
    y = np.concatenate([f.process(raw[2 * a:2 * b]) for a, b in zip(cuts[:-1], cuts[1:])])
    assert f.last_algorithm() == _lib.FIR_MATRIX
    assert f.last_kernel() == _lib.FIR_KERNEL_INT8, f.last_kernel()
    assert_parity(y, ref, what=f"K {K}")
    nch, nb = 3, 4096 + 8
    x = rng.integers(0, 256, size=(nch, 2 * nb), dtype=np.uint8)
    bank = sdr.filter.FirBank(taps, nch, sample_kind=_lib.CU8, decim=D)
    yb = bank.process(x)
    assert bank.last_kernel() == _lib.FIR_KERNEL_INT8, bank.last_kernel()
    for c in range(nch):
        assert_parity(yb[c], oracle.Fir(taps, D, sample_kind=1).process(oracle.u8_to_c64(x[c])),
                      what=f"bank K {K} ch {c}")


@pytest.mark.slow
def test_cu8_full_size_configs1_properties(sdr, oracle):
    """configs[1] fed from rtl_tcp u8 at full size (2^28 samples, the int8 kernel): windows at
    the stream ends, at per-workgroup unit boundaries and at random places against the oracle;
    then the whole stream again as two ragged blocks -- the int8 kernel sums exact integers,
    so its outputs do not depend on where tiles and blocks fall: array_equal over all 2^26."""
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer
    import scipy.signal as ss
    n = 1 << 28
    taps = ss.firwin(255, 0.2).astype(np.float32)
    dx = DeviceBuffer.empty(2 * n, np.uint8)
    chunk = 1 << 25
    for i in range(0, 2 * n, chunk):
        dx.upload(np.random.default_rng(300 + i // chunk).integers(0, 256, chunk, dtype=np.uint8),
                  offset_bytes=i)
    n_out = n // 4
    f = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    dy = DeviceBuffer.empty(n_out, np.complex64)
    assert f.process_dev(dx.ptr, n, dy.ptr, n_out) == n_out
    f.sync()
    rng = np.random.default_rng(1)
    # units: runs of 8 tiles of 256 outputs, 2048-output steps; a workgroup's range ends at
    # units * b / 256 for b = 1 .. 255 (fir_mxi_launch's blocked dealing at 256 CUs)
    units = n_out // 2048
    edges = [2048 * (units * b // 256) for b in (1, 97, 255)]
    starts = [0, n_out - 4096] + [e - 2048 for e in edges] + [int(v) for v in rng.integers(1, n_out - 4096, 4)]
    for m0 in starts:
        g0 = max(0, 4 * m0 - 256)
        g1 = 4 * (m0 + 4096)
        raw = dx.download(2 * (g1 - g0), dtype=np.uint8, offset_bytes=2 * g0)
        ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
        skip = m0 - g0 // 4
        assert_parity(dy.download(4096, offset_bytes=8 * m0), ref[skip:skip + 4096],
                      what=f"window {m0}")
    cut = 123456789  # ragged: not a tile, unit or decimation-phase boundary
    tail = DeviceBuffer(2 * (n - cut))  # the second block in its own (16-byte aligned) buffer,
    tail.copy_from(dx, 2 * (n - cut), src_off=2 * cut)  # so it takes the int8 kernel too
    g = sdr.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    dz = DeviceBuffer.empty(n_out, np.complex64)
    m1 = g.process_dev(dx.ptr, cut, dz.ptr, n_out)
    m2 = g.process_dev(tail.ptr, n - cut, dz.ptr + 8 * m1, n_out - m1)
    g.sync()
    assert m1 + m2 == n_out
    for m in range(0, n_out, 1 << 24):
        c = min(1 << 24, n_out - m)
        assert np.array_equal(dz.download(c, offset_bytes=8 * m), dy.download(c, offset_bytes=8 * m))
