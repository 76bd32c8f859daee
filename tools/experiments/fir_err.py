"""Accuracy of a FIR library variant (run through run_with_lib.py): max|err|/rms and L2 error
of configs[1]'s FIR-decimate against the oracle on a white-noise block and on bench.py's
synthetic tone pattern (2^20 samples each), both D = 4 and the D = 1 bank shape."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import pyoracle  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402

taps = ss.firwin(255, 0.2).astype(np.float32)
rng = np.random.default_rng(0)
n = 1 << 20
white = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
tones = bench.synth_iq_pattern(n, seed=1000)
for D in (4, 1):
    for name, x in (("white", white), ("tones", tones)):
        y = sdrgpu.filter.Fir(taps, decim=D, sample_kind=sdrgpu.C64).design(2.4e6).process(x)
        ref = pyoracle.Fir(taps, D, sample_kind=1).process(x).astype(np.complex128)
        d = y.astype(np.complex128) - ref
        rms = float(np.sqrt(np.mean(np.abs(ref) ** 2)))
        print(f"D={D} {name}: max|err|/rms {np.max(np.abs(d)) / rms:.3e}  "
              f"L2 {np.linalg.norm(d) / np.linalg.norm(ref):.3e}", flush=True)
