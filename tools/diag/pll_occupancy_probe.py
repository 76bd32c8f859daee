"""Per-lane rate of the time-parallel PLL's pass-1 kernel at low and full occupancy (round 5
diagnostic): the same plan (segments of 16 Ki, warm-up 8) over 64 channels (64 x 64 lanes, 64
SIMDs busy) and 1024 channels (every SIMD busy), and the serial kernels' rates, from a rocprof
kernel trace of this script.  python tools/diag/pll_occupancy_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer, synchronize  # noqa: E402

f = sdrgpu.filter
n = 1 << 20
rng = np.random.default_rng(3)
for nch in (64, 1024):
    d = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity, f.BiquadD.LowPass(20000.0, 0.7))
    pll = d.design(1.8e6, nch=nch)
    pll.set_time_parallel(16384, 8)
    ph = np.cumsum(rng.standard_normal((nch, n)).astype(np.float32) * 0.05, axis=1)
    x = DeviceBuffer.from_numpy(np.exp(1j * ph).astype(np.complex64))
    out = DeviceBuffer.empty(nch * n, np.float32)
    lk = DeviceBuffer.empty(nch * n, np.uint8)
    for _ in range(2):
        pll.reset()
        pll.process_dev(x.ptr, n, n, out.ptr, lk.ptr, n)
        synchronize()
    print(nch, pll.last_time_parallel(), flush=True)
