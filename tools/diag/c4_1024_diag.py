"""Diagnose a configs[3] chain mismatch (tests/test_firbank_gpu.py nch1024 case): run the
test's exact flow, and on a PLL mismatch save the first diverging channel's bank output, the
GPU and oracle PLL outputs / lock flags and the first differing sample to
gpurun_out/c4diag.npz, then re-run the PLL alone on that saved input (vec and scalar kernels)."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import pyoracle as oracle  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer  # noqa: E402
from test_pll_gpu import RATE, fm_channels, main_rs_design, oracle_params  # noqa: E402

nch, n, cut = 1024, 9000, int(sys.argv[1]) if len(sys.argv) > 1 else 3002
mode = sys.argv[2] if len(sys.argv) > 2 else "chain"  # chain | serial (PLL synced before the next bank block) | pllonly
rng = np.random.default_rng(45 + nch)
x = fm_channels(rng, nch, n)
taps = ss.firwin(255, 0.2).astype(np.float32)
b = sdrgpu.filter.FirBank(taps, nch, sample_kind=1)
pll = main_rs_design(sdrgpu).design(RATE, nch=nch)
dx = DeviceBuffer.from_numpy(x)
dy = DeviceBuffer.empty(nch * n, np.complex64)
do = DeviceBuffer.empty(nch * n, np.float32)
dl = DeviceBuffer.empty(nch * n, np.uint8)
if mode == "pllonly":  # bank over the whole rows first, then the PLL in the two blocks
    assert b.process_dev(dx.ptr, n, n, dy.ptr, n) == n
    b.sync()
from sdrgpu.device import synchronize  # noqa: E402
dz = DeviceBuffer.empty(nch * n, np.complex64) if mode == "otherbuf" else None
for a, e in ((0, cut), (cut, n)):
    if mode != "pllonly":
        tgt = dz if (mode == "otherbuf" and a > 0) else dy
        assert b.process_dev(dx.ptr + 8 * a, n, e - a, tgt.ptr + 8 * a, n) == e - a
        b.sync()
        if mode == "devsync":
            synchronize(0)
        if mode == "otherbuf" and a > 0:  # block 2 went to dz: copy its columns into dy afterwards
            pass
    pll.process_dev(dy.ptr + 8 * a, n, e - a, do.ptr + 4 * a, dl.ptr + a, n)
    if mode in ("serial", "pllonly"):
        pll.sync()
pll.sync()
if mode == "otherbuf":  # dy's block-2 columns from dz (row by row) so the oracle sees what the PLL read
    yz = dz.download().reshape(nch, n)
    yy = dy.download().reshape(nch, n)
    yy[:, cut:] = yz[:, cut:]
    dy.upload(np.ascontiguousarray(yy.reshape(-1)))
y = dy.download().reshape(nch, n)
out = do.download(dtype=np.float32).reshape(nch, n)
lk = dl.download(dtype=np.uint8).reshape(nch, n)
ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), y, nthreads=16)
bad = np.nonzero(((out != ref_out) & ~(np.isnan(out) & np.isnan(ref_out))) | (lk != ref_lk))
print("mode", mode, "cut", cut, "mismatching samples", bad[0].size, "channels", np.unique(bad[0])[:20])
if bad[0].size:
    c = int(bad[0][0])
    first = int(bad[1][bad[0] == c].min())
    print("first channel", c, "first sample", first, "gpu", out[c, first], lk[c, first], "ref", ref_out[c, first], ref_lk[c, first])
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "c4diag.npz"), y=y[c], out=out[c], lk=lk[c], ref_out=ref_out[c],
             ref_lk=ref_lk[c], c=c, first=first, cut=cut)
    # the same channel alone through the PLL, one block (vec path) and as the two blocks
    for blocks in ((0, n), (0, cut, n)):
        p1 = main_rs_design(sdrgpu).design(RATE, nch=1)
        d1 = DeviceBuffer.from_numpy(np.ascontiguousarray(y[c]))
        o1 = DeviceBuffer.empty(n, np.float32)
        l1 = DeviceBuffer.empty(n, np.uint8)
        for a, e in zip(blocks[:-1], blocks[1:]):
            p1.process_dev(d1.ptr + 8 * a, n, e - a, o1.ptr + 4 * a, l1.ptr + a, n)
        p1.sync()
        g1, k1 = o1.download(dtype=np.float32), l1.download(dtype=np.uint8)
        print("single-channel", blocks, "vs oracle: out diff", int(np.sum(g1 != ref_out[c])),
              "lock diff", int(np.sum(k1 != ref_lk[c])), "vs 1024-ch run: out diff", int(np.sum(g1 != out[c])))
