"""configs[3] chain: does dy[:, :cut] change while PLL block 1 runs beside bank block 2?
Snapshot dy after bank block 1, run the chain, snapshot again; compare, and compare the GPU PLL
with the oracle fed each snapshot."""
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

nch, n = 1024, 9000
cut = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
pad = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # extra MiB allocated before dy (address shift)
scalar = len(sys.argv) > 3 and sys.argv[3] == "scalar"  # lock flags at an odd address: the PLL's LDS-free pll_kernel<..., false>
rng = np.random.default_rng(45 + nch)
x = fm_channels(rng, nch, n)
taps = ss.firwin(255, 0.2).astype(np.float32)
b = sdrgpu.filter.FirBank(taps, nch, sample_kind=1)
pll = main_rs_design(sdrgpu).design(RATE, nch=nch)
dx = DeviceBuffer.from_numpy(x)
spacer = DeviceBuffer(pad << 20) if pad else None
dy = DeviceBuffer.empty(nch * n, np.complex64)
dy.fill_zero()
do = DeviceBuffer.empty(nch * n, np.float32)
dl = DeviceBuffer.empty(nch * n + 8, np.uint8)
lko = 1 if scalar else 0
assert b.process_dev(dx.ptr, n, cut, dy.ptr, n) == cut
b.sync()
y1 = dy.download().reshape(nch, n)
pll.process_dev(dy.ptr, n, cut, do.ptr, dl.ptr + lko, n)
assert b.process_dev(dx.ptr + 8 * cut, n, n - cut, dy.ptr + 8 * cut, n) == n - cut
b.sync()
pll.sync()
y2 = dy.download().reshape(nch, n)
ch = (y1[:, :cut] != y2[:, :cut])
rows, cols = np.nonzero(ch)
print("scalar PLL" if scalar else "split PLL", "pad", pad, "MiB  dy[:, :cut] changed during the chain:", int(ch.sum()), "rows", np.unique(rows)[:24],
      "cols", np.unique(cols)[:16])
if rows.size:
    r, c = rows[0], cols[0]
    print(" e.g. row", r, "col", c, "after block 1", y1[r, c], "after the chain", y2[r, c])
out = do.download(dtype=np.float32).reshape(nch, n)[:, :cut]
lk = dl.download(dtype=np.uint8)[lko:lko + nch * n].reshape(nch, n)[:, :cut]
for name, yy in (("snapshot after block 1", y1), ("final dy", y2)):
    ro, rl = oracle.pll_batch(oracle_params(oracle), np.ascontiguousarray(yy[:, :cut]), nthreads=16)
    bad = (out != ro) | (lk != rl)
    print(" GPU PLL block 1 vs oracle on the", name + ":", int(bad.sum()), "samples in", np.unique(np.nonzero(bad)[0]).size, "channels")
    if bad.any() and name == "final dy":
        chs = np.unique(np.nonzero(bad)[0])
        first = np.array([np.argmax(bad[c]) for c in chs])
        fo = np.array([np.argmax(out[c] != ro[c]) if (out[c] != ro[c]).any() else -1 for c in chs])
        fl = np.array([np.argmax(lk[c] != rl[c]) if (lk[c] != rl[c]).any() else -1 for c in chs])
        print("  bad channels:", chs.tolist())
        print("  first bad sample per channel (min/median/max):", int(first.min()), int(np.median(first)), int(first.max()),
              " histogram by 8-sample chunk:", np.bincount(first // 8).nonzero()[0][:20].tolist())
        print("  first out mismatch:", fo[:16].tolist(), " first lock mismatch:", fl[:16].tolist())
        c0 = chs[0]; i0 = first[0]
        print("  e.g. ch", int(c0), "samples", int(i0), "..", int(i0) + 4, "gpu", out[c0, i0:i0 + 4].tolist(), "oracle", ro[c0, i0:i0 + 4].tolist())
