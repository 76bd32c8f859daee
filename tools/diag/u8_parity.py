"""u8 FIR parity spot check for library variants (run under tools/experiments/run_with_lib.py):
configs[1]-shaped fused u8 streams against the oracle, ragged blocks and a 5-channel bank."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import pyoracle as oracle  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402

worst = 0.0
rng = np.random.default_rng(3)
for K, n, cuts in ((255, 1 << 21, (0, 777, 300001, 1 << 21)), (97, 200003, (0, 200003))):
    taps = ss.firwin(K, 0.2).astype(np.float32)
    raw = rng.integers(0, 256, size=2 * n, dtype=np.uint8)
    ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(raw))
    f = sdrgpu.filter.Fir(taps, decim=4, sample_kind=_lib.CU8).design(2.4e6)
    y = np.concatenate([f.process(raw[2 * a:2 * b]) for a, b in zip(cuts[:-1], cuts[1:])])
    err = float(np.max(np.abs(y - ref)) / np.sqrt(np.mean(np.abs(ref) ** 2)))
    worst = max(worst, err)
    print(f"K {K} n {n} blocks {len(cuts) - 1}: max err / rms {err:.2e}")
for K, n, D in ((255, 1 << 20, 1), (61, 100003, 1), (255, 1 << 20, 8), (255, 1 << 20, 2)):
    taps = ss.firwin(K, 0.2).astype(np.float32)
    raw = rng.integers(0, 256, size=2 * n, dtype=np.uint8)
    ref = oracle.Fir(taps, D, sample_kind=1).process(oracle.u8_to_c64(raw))
    f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=_lib.CU8).design(2.4e6)
    y = np.concatenate([f.process(raw[:2 * 4097]), f.process(raw[2 * 4097:])])
    err = float(np.max(np.abs(y - ref)) / np.sqrt(np.mean(np.abs(ref) ** 2)))
    worst = max(worst, err)
    print(f"D {D} K {K} n {n}: max err / rms {err:.2e}")
nch, nb = 5, 40000
taps = ss.firwin(255, 0.2).astype(np.float32)
x = rng.integers(0, 256, size=(nch, 2 * nb), dtype=np.uint8)
y = sdrgpu.filter.FirBank(taps, nch, sample_kind=_lib.CU8, decim=4).process(x)
for c in range(nch):
    ref = oracle.Fir(taps, 4, sample_kind=1).process(oracle.u8_to_c64(x[c]))
    worst = max(worst, float(np.max(np.abs(y[c] - ref)) / np.sqrt(np.mean(np.abs(ref) ** 2))))
print("u8 parity", "OK" if worst < 1e-5 else "FAIL", f"worst {worst:.2e}")
sys.exit(0 if worst < 1e-5 else 1)
