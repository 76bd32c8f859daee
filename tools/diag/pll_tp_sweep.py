"""Time-parallel PLL at configs[3]'s shape (bench_configs c4's data: synthetic IQ through the
255-tap matched-filter bank, then the main.rs PLL, 1024 ch x 2^20): PLL time and recomputed
segments per (segment, warm-up) pair, plus a 4-channel whole-stream check against the oracle.
python tools/diag/pll_tp_sweep.py seg:warm ..."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unnamed-rust-sdr_amd"), os.path.join(ROOT, "oracle")]
import bench_configs as bc  # noqa: E402
import pyoracle  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer, synchronize  # noqa: E402

f = sdrgpu.filter
nch, n, rate = 1024, 1 << 20, 1.8e6
taps = ss.firwin(255, 0.2).astype(np.float32)
bank = f.FirBank(taps, nch, sample_kind=sdrgpu.C64)
x = DeviceBuffer.empty(nch * n)
bc.fill(x, nch * n, 4)
mf = DeviceBuffer.empty(nch * n)
out = DeviceBuffer.empty(nch * n, np.float32)
lk = DeviceBuffer.empty(nch * n, np.uint8)
bank.process_dev(x.ptr, n, n, mf.ptr, n)
bank.sync()
p = pyoracle.pll_params(0.0, 0.035, rate, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
chans = [0, 341, 513, 1023]
mfs = np.stack([mf.download(n, offset_bytes=8 * c * n) for c in chans])
ref_out, ref_lk = pyoracle.pll_batch(p, mfs, nthreads=4)
for arg in sys.argv[1:]:
    seg, warm = (int(v) for v in arg.split(":"))
    pll = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                      f.BiquadD.LowPass(20000.0, 0.7)).design(rate, nch=nch)
    pll.set_stream(bank.stream())
    pll.set_time_parallel(seg, warm)

    def run():
        pll.reset()
        pll.process_dev(mf.ptr, n, n, out.ptr, lk.ptr, n)

    _, ms = bc.time_events(run, bank.stream(), 3, 1, lambda: (bank.sync(), synchronize()))
    segs, rec = pll.last_time_parallel()
    go = np.stack([out.download(n, dtype=np.float32, offset_bytes=4 * c * n) for c in chans])
    gl = np.stack([lk.download(n, dtype=np.uint8, offset_bytes=c * n) for c in chans])
    bad = int(np.sum(go != ref_out) + np.sum(gl != ref_lk))
    print(f"seg {seg:6d} warm {warm:6d}: {ms:8.3f} ms ({ms * 1e6 / n:6.2f} ns/sample), {segs} segments,"
          f" {rec} recomputed, check {'OK' if bad == 0 else f'{bad} WRONG'}", flush=True)
