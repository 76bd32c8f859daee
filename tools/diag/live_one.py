"""One examples/live.rs-shaped STFT launch sequence (1000-point frames, hop 500, fused dB) over
2^26 c64 samples, 5 launches: a short target for rocprofv3 --pmc passes.  Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer, synchronize  # noqa: E402

n_in = 1 << 26
rng = np.random.default_rng(3)
x = (rng.standard_normal(1 << 22) + 1j * rng.standard_normal(1 << 22)).astype(np.complex64)
s = sdrgpu.fft.Stft(1000, 500, output=os.environ.get("LIVE_OUT", "db"))
dx = DeviceBuffer(n_in * 8)
for off in range(0, n_in * 8, x.nbytes):
    dx.upload(x, offset_bytes=off)
nf = s.output_len(n_in)
dy = DeviceBuffer(nf * 1000 * 8)
for _ in range(5):
    s.reset()
    s.process_dev(dx.ptr, n_in, dy.ptr, nf)
synchronize()
print("done", nf)
