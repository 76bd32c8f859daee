"""Time-parallel PLL on an unlocked loop (round 6): 1024 channels x 2^20 samples of
complex white noise (no carrier) through the main.rs PLL design, automatic plan vs one serial
pass: per-block times, the segments recomputed, the three phase times, and the adapted plan on
the following blocks; outputs of the two handles compared bit for bit.
    python tools/diag/pll_noise_timing.py [log2n]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import bench_configs as bc  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer, synchronize  # noqa: E402

f = sdrgpu.filter
nch, rate = 1024, 1.8e6
n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 20)
rng = np.random.default_rng(7)
x = DeviceBuffer.from_numpy(((rng.standard_normal((nch, n)) + 1j * rng.standard_normal((nch, n))) * 0.1)
                            .astype(np.complex64))
outs = []
for mode in ("auto", "serial"):
    pll = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                      f.BiquadD.LowPass(20000.0, 0.7)).design(rate, nch=nch)
    if mode == "serial":
        pll.set_time_parallel(-1)
    pll.set_phase_timing(True)
    out = DeviceBuffer.empty(nch * n, np.float32)
    lk = DeviceBuffer.empty(nch * n, np.uint8)
    for blk in range(2 if mode == "auto" else 1):
        _, ms = bc.time_events(lambda: pll.process_dev(x.ptr, n, n, out.ptr, lk.ptr, n), pll.stream(), 1, 0,
                               lambda: (pll.sync(), synchronize()))
        segs, rec = pll.last_time_parallel()
        print(f"{mode} block {blk}: {ms:8.3f} ms  segments/channel {segs}  recomputed {rec} of {segs * nch}"
              f"  phases (pass 1, re-run, walk) ms {tuple(round(v, 3) for v in pll.last_phase_ms())}", flush=True)
        if blk == 0:
            outs.append((out.download(dtype=np.float32), lk.download(dtype=np.uint8)))
print("block 0 outputs and lock flags identical (auto vs serial):",
      bool(np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])))
