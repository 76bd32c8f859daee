"""Diagnose the C4 bank -> PLL chain: where do PLL outputs differ from the oracle fed the
final bank output, and does the bank's first-block output change after the second block?"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "unnamed-rust-sdr_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import sdrgpu as sdr
from sdrgpu import _lib
from sdrgpu.device import DeviceBuffer
import scipy.signal as ss
import pyoracle as oracle
from test_pll_gpu import RATE, fm_channels, main_rs_design, oracle_params

rng = np.random.default_rng(45)
nch, n = 128, 16384
x = fm_channels(rng, nch, n)
taps = ss.firwin(255, 0.2).astype(np.float32)
b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_AUTO)
dx = DeviceBuffer.from_numpy(x)
dy = DeviceBuffer.empty(nch * n, np.complex64)
snap = []
for a, e in ((0, 6000), (6000, n)):
    b.process_dev(dx.ptr + 8 * a, n, e - a, dy.ptr + 8 * a, n)
    b.sync()
    snap.append(dy.download().reshape(nch, n).copy())
y = snap[1]
d01 = snap[0][:, :6000] != y[:, :6000]
print("block-1 region changed by block 2:", int(d01.sum()))
ref = oracle.fir_batch(taps, x, 1, nthreads=16)
err = np.abs(y.astype(np.complex128) - ref)
rms = np.sqrt(np.mean(np.abs(ref) ** 2, axis=1))
print("worst max/rms", float((err.max(axis=1) / rms).max()))
for rep in range(3):
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    do = DeviceBuffer.empty(nch * n, np.float32)
    dl = DeviceBuffer.empty(nch * n, np.uint8)
    dyy = DeviceBuffer.from_numpy(y)
    for a, e in ((0, 6000), (6000, n)):
        pll.process_dev(dyy.ptr + 8 * a, n, e - a, do.ptr + 4 * a, dl.ptr + a, n)
    pll.sync()
    out = do.download(dtype=np.float32).reshape(nch, n)
    lk = dl.download(dtype=np.uint8).reshape(nch, n)
    ro, rl = oracle.pll_batch(oracle_params(oracle), y, nthreads=16)
    bad = (out != ro) | (lk != rl)
    print(f"rep {rep}: pll mismatches {int(bad.sum())} channels {np.unique(np.nonzero(bad)[0])[:10]}"
          f" first col {np.nonzero(bad)[1].min() if bad.any() else -1}")

# exactly the test's interleaving: PLL block 1 runs on its stream while bank block 2 runs
for rep in range(4):
    b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_AUTO)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    dy = DeviceBuffer.empty(nch * n, np.complex64)
    do = DeviceBuffer.empty(nch * n, np.float32)
    dl = DeviceBuffer.empty(nch * n, np.uint8)
    for a, e in ((0, 6000), (6000, n)):
        b.process_dev(dx.ptr + 8 * a, n, e - a, dy.ptr + 8 * a, n)
        b.sync()
        pll.process_dev(dy.ptr + 8 * a, n, e - a, do.ptr + 4 * a, dl.ptr + a, n)
    pll.sync()
    y2 = dy.download().reshape(nch, n)
    out = do.download(dtype=np.float32).reshape(nch, n)
    lk = dl.download(dtype=np.uint8).reshape(nch, n)
    ro, rl = oracle.pll_batch(oracle_params(oracle), y2, nthreads=16)
    bad = (out != ro) | (lk != rl)
    cols = np.nonzero(bad)[1]
    print(f"interleaved rep {rep}: y same as before {np.array_equal(y2, y)}; pll mismatches {int(bad.sum())}"
          f" channels {np.unique(np.nonzero(bad)[0])[:10]} cols {cols.min() if bad.any() else -1}.."
          f"{cols.max() if bad.any() else -1}")

def variant(name, sync_between, separate_input, reps=6):
    dyy = DeviceBuffer.from_numpy(y)
    nbad = []
    for rep in range(reps):
        b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_AUTO)
        pll = main_rs_design(sdr).design(RATE, nch=nch)
        dy = DeviceBuffer.empty(nch * n, np.complex64)
        do = DeviceBuffer.empty(nch * n, np.float32)
        dl = DeviceBuffer.empty(nch * n, np.uint8)
        src = dyy if separate_input else dy
        for a, e in ((0, 6000), (6000, n)):
            b.process_dev(dx.ptr + 8 * a, n, e - a, dy.ptr + 8 * a, n)
            b.sync()
            pll.process_dev(src.ptr + 8 * a, n, e - a, do.ptr + 4 * a, dl.ptr + a, n)
            if sync_between:
                pll.sync()
        pll.sync()
        out = do.download(dtype=np.float32).reshape(nch, n)
        lk = dl.download(dtype=np.uint8).reshape(nch, n)
        ro, rl = oracle.pll_batch(oracle_params(oracle), y, nthreads=16)
        bad = (out != ro) | (lk != rl)
        nbad.append((int(bad.sum()), list(np.unique(np.nonzero(bad)[0])[:3])))
    print(name, nbad)

def variant_d(reps=8):
    res = []
    for rep in range(reps):
        b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_AUTO)
        pll = main_rs_design(sdr).design(RATE, nch=nch)
        dy = DeviceBuffer.empty(nch * n, np.complex64)
        for a, e in ((0, 6000), (6000, n)):
            b.process_dev(dx.ptr + 8 * a, n, e - a, dy.ptr + 8 * a, n)
        b.sync()
        st = [pll.state(c) for c in range(nch)]
        nz = [c for c, v in enumerate(st) if v != (0.0, 0j)]
        res.append(nz[:4] + ([len(nz)] if nz else []))
    print("D state after bank only:", res)

def detail(reps=12):
    for rep in range(reps):
        b = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_AUTO)
        pll = main_rs_design(sdr).design(RATE, nch=nch)
        dy = DeviceBuffer.empty(nch * n, np.complex64)
        do = DeviceBuffer.empty(nch * n, np.float32)
        dl = DeviceBuffer.empty(nch * n, np.uint8)
        do.fill_zero(); dl.fill_zero()
        for a, e in ((0, 6000), (6000, n)):
            b.process_dev(dx.ptr + 8 * a, n, e - a, dy.ptr + 8 * a, n)
            b.sync()
            pll.process_dev(dy.ptr + 8 * a, n, e - a, do.ptr + 4 * a, dl.ptr + a, n)
        pll.sync()
        out = do.download(dtype=np.float32).reshape(nch, n)
        lk = dl.download(dtype=np.uint8).reshape(nch, n)
        ro, rl = oracle.pll_batch(oracle_params(oracle), y, nthreads=16)
        bad = (out != ro) | (lk != rl)
        if not bad.any():
            print(f"detail rep {rep}: ok"); continue
        chs = np.unique(np.nonzero(bad)[0])
        c = chs[0]
        cols = np.nonzero(bad[c])[0]
        print(f"detail rep {rep}: {int(bad.sum())} bad, chans {list(chs)}")
        print(f"  ch {c}: first bad col {cols[0]} ncols {len(cols)} lk bad {int((lk[c]!=rl[c]).sum())} out bad {int((out[c]!=ro[c]).sum())}")
        j = cols[0]
        print("  got", out[c, j-2:j+6], lk[c, j-2:j+6])
        print("  ref", ro[c, j-2:j+6], rl[c, j-2:j+6])
        print("  final state got", pll.state(int(c)))
        # oracle on the prefix to the same column: does the kernel's trajectory match a
        # shifted or perturbed input?
def cocheck(label, other, reps=10):
    """PLL block 1 runs while `other()` (another kernel on another stream) runs."""
    res = []
    for rep in range(reps):
        pll = main_rs_design(sdr).design(RATE, nch=nch)
        do = DeviceBuffer.empty(nch * n, np.float32)
        dl = DeviceBuffer.empty(nch * n, np.uint8)
        dyy = DeviceBuffer.from_numpy(y)
        pll.process_dev(dyy.ptr, n, n, do.ptr, dl.ptr, n)
        other()
        pll.sync()
        out = do.download(dtype=np.float32).reshape(nch, n)
        lk = dl.download(dtype=np.uint8).reshape(nch, n)
        bad = (out != ro) | (lk != rl)
        res.append((int(bad.sum()), [int(c) for c in np.unique(np.nonzero(bad)[0])[:2]]))
    print(label, res)

ro, rl = oracle.pll_batch(oracle_params(oracle), y, nthreads=16)
big = DeviceBuffer.from_numpy((np.random.default_rng(0).standard_normal(2 * (1 << 24)).astype(np.float32)).view(np.complex64))
bigo = DeviceBuffer.empty(1 << 24, np.complex64)
f4 = sdr.filter.Fir(taps, decim=4, sample_kind=1).design(2.4e6)
bk = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_AUTO)
bko = sdr.filter.FirBank(taps, nch, sample_kind=1, decim=1, algorithm=_lib.FIR_OVERLAP_SAVE)
dyb = DeviceBuffer.empty(nch * n, np.complex64)
cocheck("alone", lambda: None)
cocheck("with D4 mxh", lambda: (f4.process_dev(big.ptr, 1 << 24, bigo.ptr, 1 << 24), f4.sync()))
cocheck("with D1 bank mxh", lambda: (bk.process_dev(dx.ptr, n, n, dyb.ptr, n), bk.sync()))
cocheck("with D1 bank os", lambda: (bko.process_dev(dx.ptr, n, n, dyb.ptr, n), bko.sync()))
