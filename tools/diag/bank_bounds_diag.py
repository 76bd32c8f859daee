"""Does a FIR bank block write outside its [a, e) column range?  configs[3]'s shape (1024
channels, ld 9000): after block 1, fill every row's [0, cut) with a NaN sentinel, run block 2
and look for changed sentinel bytes; also time-order check the PLL reads."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd"), os.path.join(ROOT, "tests")]
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer  # noqa: E402
from test_pll_gpu import fm_channels  # noqa: E402

nch, n = 1024, 9000
cut = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
rng = np.random.default_rng(45 + nch)
x = fm_channels(rng, nch, n)
taps = ss.firwin(255, 0.2).astype(np.float32)
b = sdrgpu.filter.FirBank(taps, nch, sample_kind=1)
dx = DeviceBuffer.from_numpy(x)
dy = DeviceBuffer.empty(nch * n, np.complex64)
guard = DeviceBuffer.from_numpy(np.full(4096, np.nan, np.complex64))  # allocation right after dy
assert b.process_dev(dx.ptr, n, cut, dy.ptr, n) == cut
b.sync()
y1 = dy.download().reshape(nch, n)
sent = y1.copy()
sent[:, :cut] = np.complex64(complex(np.nan, 1.0))
sent[:, cut:] = np.complex64(complex(np.nan, 2.0))
dy.upload(np.ascontiguousarray(sent.reshape(-1)))
assert b.process_dev(dx.ptr + 8 * cut, n, n - cut, dy.ptr + 8 * cut, n) == n - cut
b.sync()
y2 = dy.download().reshape(nch, n)
before = y2[:, :cut].view(np.uint64) != sent[:, :cut].view(np.uint64)
after_untouched = np.isnan(y2[:, cut:].real)
print("cut", cut, "block-2 writes into [0, cut):", int(before.sum()), "rows", np.unique(np.nonzero(before)[0])[:16],
      "| outputs of block 2 left unwritten:", int(after_untouched.sum()),
      "| guard changed:", int(np.sum(~np.isnan(guard.download().real))))
