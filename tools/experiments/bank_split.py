"""configs[4] bank (8192 ch x 2^16, 255 taps, D = 1): one launch over all channels vs the
same channels as S independent half/quarter banks launched on S streams at once (timing
only; each FirBank is its own stream)."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "unnamed-rust-sdr_amd"))
import numpy as np
import scipy.signal as ss
import sdrgpu
from sdrgpu.device import DeviceBuffer, synchronize

taps = ss.firwin(255, 0.2).astype(np.float32)
nch, n = 8192, 1 << 16
x = DeviceBuffer.empty(nch * n, np.complex64)
rng = np.random.default_rng(1)
blk = (rng.standard_normal(1 << 22) + 1j * rng.standard_normal(1 << 22)).astype(np.complex64) * np.float32(0.3)
for off in range(0, nch * n, 1 << 22):
    x.upload(blk, offset_bytes=8 * off)
y = DeviceBuffer.empty(nch * n, np.complex64)
for S in (1, 2, 4, 1, 2, 4):
    per = nch // S
    banks = [sdrgpu.filter.FirBank(taps, per, sample_kind=sdrgpu.C64) for _ in range(S)]
    def step():
        for i, b in enumerate(banks):
            b.process_dev(x.ptr + 8 * i * per * n, n, n, y.ptr + 8 * i * per * n, n)
    for _ in range(3):
        step()
    for b in banks:
        b.sync()
    synchronize(0)
    t0 = time.perf_counter()
    reps = 20
    for _ in range(reps):
        step()
    for b in banks:
        b.sync()
    synchronize(0)
    ms = (time.perf_counter() - t0) / reps * 1e3
    print(f"S={S}: {ms:.3f} ms per 8192-channel step ({nch * n / ms / 1e6 * 1e3 / 1e3:.1f} Gsps)", flush=True)
