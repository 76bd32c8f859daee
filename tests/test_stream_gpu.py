"""Async host streaming: sdrgpu_fir_process_async from pinned host blocks
(the Block adapter's producer/consumer split, reference src/signal/adapters/block.rs:105-207)
gives exactly the outputs of the synchronous host path on the same stream of blocks."""
import numpy as np
import pytest
import scipy.signal as ss

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["c64", "u8"])
def test_fir_process_async_matches_sync(sdr, oracle, kind):
    from sdrgpu.device import PinnedBuffer
    taps = ss.firwin(255, 0.2).astype(np.float32)
    sk = sdr.C64 if kind == "c64" else sdr.CU8
    ib = 8 if kind == "c64" else 2
    rng = np.random.default_rng(17)
    sizes = [40000, 4, 65536, 12345, 99997, 8]
    a = sdr.filter.Fir(taps, decim=4, sample_kind=sk).design(2.4e6)
    b = sdr.filter.Fir(taps, decim=4, sample_kind=sk).design(2.4e6)
    ins = [PinnedBuffer(max(sizes) * ib, np.uint8) for _ in range(2)]
    outs = [PinnedBuffer(max(sizes) // 4 + 2, np.complex64) for _ in range(2)]
    ref, got, pend = [], [], []
    for i, n in enumerate(sizes):
        raw = rng.integers(0, 256, size=n * ib, dtype=np.uint8)
        if kind == "c64":
            raw = (rng.standard_normal(2 * n).astype(np.float32) * 0.3).view(np.uint8)
        ref.append(b.process(raw.view(np.complex64) if kind == "c64" else raw))
        if len(pend) == 2:  # both slots in flight: wait, then collect the older one
            a.sync()
            for j, m in pend:
                got.append(outs[j].array[:m].copy())
            pend = []
        slot = i & 1
        ins[slot].array[:n * ib] = raw
        m = a.process_async(ins[slot].ptr, n, outs[slot].ptr, outs[slot].n)
        pend.append((slot, m))
    a.sync()
    for j, m in pend:
        got.append(outs[j].array[:m].copy())
    for r, g in zip(ref, got):
        assert np.array_equal(r, g)
    for p in ins + outs:
        p.free()


@pytest.mark.parametrize("kind", ["c64", "u8"])
def test_stft_process_async_matches_sync(sdr, kind):
    from sdrgpu import _lib
    from sdrgpu.device import PinnedBuffer
    n, hop = 4096, 1024
    sk = _lib.C64 if kind == "c64" else _lib.CU8
    ib = 8 if kind == "c64" else 2
    rng = np.random.default_rng(19)
    sizes = [40000, 3, 65536, 1023, 20001]
    a = sdr.fft.Stft(n, hop, input_kind=sk)
    b = sdr.fft.Stft(n, hop, input_kind=sk)
    ins = [PinnedBuffer(max(sizes) * ib, np.uint8) for _ in range(2)]
    outs = [PinnedBuffer((max(sizes) // hop + 2) * n, np.complex64) for _ in range(2)]
    ref, got, pend = [], [], []
    for i, m in enumerate(sizes):
        raw = rng.integers(0, 256, size=m * ib, dtype=np.uint8)
        if kind == "c64":
            raw = (rng.standard_normal(2 * m).astype(np.float32)).view(np.uint8)
        ref.append(b.process(raw.view(np.complex64) if kind == "c64" else raw))
        if len(pend) == 2:
            a.sync()
            got += [outs[j].array[:nf * n].reshape(nf, n).copy() for j, nf in pend]
            pend = []
        slot = i & 1
        ins[slot].array[:m * ib] = raw
        nf = a.process_async(ins[slot].ptr, m, outs[slot].ptr, outs[slot].n // n)
        pend.append((slot, nf))
    a.sync()
    got += [outs[j].array[:nf * n].reshape(nf, n).copy() for j, nf in pend]
    for r, g in zip(ref, got):
        assert np.array_equal(r, g)
    for p in ins + outs:
        p.free()


def test_pll_process_async_matches_sync(sdr):
    from sdrgpu.device import PinnedBuffer
    from test_pll_gpu import RATE, fm_channels, main_rs_design
    rng = np.random.default_rng(23)
    nch = 48
    sizes = [5000, 1, 17, 9000, 2048]
    a = main_rs_design(sdr).design(RATE, nch=nch)
    b = main_rs_design(sdr).design(RATE, nch=nch)
    x = fm_channels(rng, nch, sum(sizes))
    ins = [PinnedBuffer(nch * max(sizes), np.complex64) for _ in range(2)]
    outs = [PinnedBuffer(nch * max(sizes), np.float32) for _ in range(2)]
    lks = [PinnedBuffer(nch * max(sizes), np.uint8) for _ in range(2)]
    ref, got, pend, off = [], [], [], 0
    for i, m in enumerate(sizes):
        blk = np.ascontiguousarray(x[:, off:off + m])
        off += m
        ref.append(b.process(blk))
        if len(pend) == 2:
            a.sync()
            got += [(outs[j].array[:nch * k].reshape(nch, k).copy(),
                     lks[j].array[:nch * k].reshape(nch, k).copy()) for j, k in pend]
            pend = []
        slot = i & 1
        ins[slot].array[:nch * m] = blk.reshape(-1)
        a.process_async(ins[slot].ptr, m, outs[slot].ptr, lks[slot].ptr)
        pend.append((slot, m))
    a.sync()
    got += [(outs[j].array[:nch * k].reshape(nch, k).copy(),
             lks[j].array[:nch * k].reshape(nch, k).copy()) for j, k in pend]
    for (ro, rl), (go, gl) in zip(ref, got):
        assert np.array_equal(ro, go) and np.array_equal(rl, gl)
    for p in ins + outs + lks:
        p.free()
