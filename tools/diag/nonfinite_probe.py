"""Which outputs go non-finite when one input sample is NaN or inf, per FIR path, against the
oracle (the reference's sequential f32 sum: the K outputs whose window holds the sample).
Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import pyoracle  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402

rng = np.random.default_rng(1)
K = 255
taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
n = 20000
base = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
for D in (4, 1, 2, 8):
    for bad in (np.nan, np.inf):
        for pos in (5000, 5003, 10240):
            x = base.copy()
            x[pos] = complex(bad, 0.0)
            ref = pyoracle.Fir(taps, D, sample_kind=1).process(x)
            rb = ~np.isfinite(ref)
            for algo, a in (("direct", _lib.FIR_DIRECT), ("os", _lib.FIR_OVERLAP_SAVE), ("mx", _lib.FIR_MATRIX)):
                try:
                    f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=1, algorithm=a).design(2.4e6)
                except _lib.SdrGpuError:
                    continue
                y = f.process(x)
                yb = ~np.isfinite(y)
                fin = rb == yb
                err = np.abs(y[~rb] - ref[~rb]).max() if (~rb).any() else 0
                print(f"D={D} {bad} @{pos} {algo:6s} kernel={f.last_kernel()} ref_nonfinite={rb.sum()} "
                      f"gpu_nonfinite={yb.sum()} same_set={bool(fin.all())} max_err_on_finite={err:.2e}", flush=True)
