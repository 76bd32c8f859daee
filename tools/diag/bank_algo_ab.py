"""configs[4] bank (8192 ch x 2^16 c64, 255 taps, D = 1) per FIR algorithm: the MFMA kernel vs
overlap-save vs direct, driver-style timing (5 warmups + 20 launches, HIP events), with a
spot check of 3 channels against the oracle.  python tools/diag/bank_algo_ab.py [algos...]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unnamed-rust-sdr_amd"), os.path.join(ROOT, "oracle")]
import bench_configs as bc  # noqa: E402
import pyoracle  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer  # noqa: E402

nch, n = 8192, 1 << 16
taps = ss.firwin(255, 0.2).astype(np.float32)
x = DeviceBuffer.empty(nch * n)
bc.fill(x, nch * n, 9)
y = DeviceBuffer.empty(nch * n)
names = sys.argv[1:] or ["mx", "os", "mx", "os"]
ids = {"mx": _lib.FIR_MATRIX, "os": _lib.FIR_OVERLAP_SAVE, "direct": _lib.FIR_DIRECT}
for name in names:
    b = sdrgpu.filter.FirBank(taps, nch, sample_kind=sdrgpu.C64, algorithm=ids[name])
    step = lambda: b.process_dev(x.ptr, n, n, y.ptr, n)
    wall, ms = bc.time_events(step, b.stream(), 20, 5, b.sync)
    b.reset()
    b.process_dev(x.ptr, n, n, y.ptr, n)
    b.sync()
    worst = 0.0
    for c in (0, 4097, nch - 1):
        xc = x.download(n, offset_bytes=8 * c * n)
        yc = y.download(n, offset_bytes=8 * c * n).astype(np.complex128)
        ref = pyoracle.Fir(taps, 1, sample_kind=1).process(xc).astype(np.complex128)
        worst = max(worst, float(np.abs(yc - ref).max() / np.sqrt(np.mean(np.abs(ref) ** 2))))
    frac = 16 * nch * n / (ms * 1e-3) / 8e12
    print(f"{name:6s} algo {b.last_algorithm()} kernel {b.last_kernel()}: {ms:.4f} ms = {frac:.3f} of 8 TB/s"
          f" (wall {wall * 1e3:.3f} ms); spot max/rms {worst:.2e}", flush=True)
