"""Where do finite outputs of the inf / NaN cases go wrong?  Runs tests/test_fir_gpu.py's
NONFINITE case 3 / 0 at D = 4, 2, 1 three times each and prints the wrong finite outputs'
indices, their 256-output tiles and whether that tile's window held a non-finite sample.
Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import pyoracle  # noqa: E402
import sdrgpu  # noqa: E402
from test_fir_gpu import NONFINITE  # noqa: E402

for case in (0, 3, 5):
    for D in (4, 2, 1):
        rng = np.random.default_rng(700 + case)
        taps = (rng.standard_normal(255) / np.sqrt(255)).astype(np.float32)
        n = 40000
        x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        for i, v in NONFINITE[case]:
            x[i] = v
        ref = pyoracle.Fir(taps, D, sample_kind=1).process(x)
        bad_in = ~np.isfinite(x.real) | ~np.isfinite(x.imag)
        for rep in range(int(os.environ.get("REPS", "3"))):
            f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=1).design(2.4e6)
            y = np.concatenate([f.process(x[:20000]), f.process(x[20000:])])
            fin = np.isfinite(ref.real) & np.isfinite(ref.imag)
            err = np.where(fin, np.abs(y - ref), 0)
            rms = np.sqrt(np.mean(np.abs(ref[fin]) ** 2))
            wrong = np.nonzero(err > 1e-5 * rms)[0]
            desc = []
            for m in wrong[:12]:
                blk = 0 if D - 1 + D * m < 20000 else 1
                mm = m if blk == 0 else m - (len(y) - len(f.process(np.zeros(0, np.complex64))))
                g = D - 1 + D * m
                win = bad_in[max(0, g - 254):g + 1].any()
                desc.append(f"m={m} g={g} tileTO={m // (256 * (4 if D == 1 else (2 if D == 2 else 1)))} "
                            f"err/rms={err[m] / rms:.2e} win_nonfinite={win} y={y[m]:.4g} ref={ref[m]:.4g}")
            print(f"case {case} D {D} rep {rep}: {len(wrong)} wrong finite outputs", flush=True)
            for d in desc:
                print("   ", d)
