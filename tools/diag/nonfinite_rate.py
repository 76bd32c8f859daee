"""Time of one FIR launch on 2^24 samples when inf / NaN samples force the exact-sum fallback
(fir_mxh exact_tile, fir_exact.hpp) into many tiles: clean input, one NaN per 1024 samples
(every tile), all NaN.  HIP events on the handle's stream, median of 5 after 2 warmups.
Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer, Event, synchronize  # noqa: E402

n = 1 << 24
rng = np.random.default_rng(5)
taps = (rng.standard_normal(255) / 16).astype(np.float32)
base = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
inputs = {"clean": base}
x = base.copy(); x[::1024] = np.nan; inputs["nan_per_1024"] = x
inputs["all_nan"] = np.full(n, complex(np.nan, np.nan), np.complex64)
paths = [("mxh D4", 4, _lib.FIR_AUTO), ("mxh D1", 1, _lib.FIR_AUTO), ("direct D4", 4, _lib.FIR_DIRECT),
         ("os D4", 4, _lib.FIR_OVERLAP_SAVE), ("bf16x3 D8", 8, _lib.FIR_AUTO)]
for name, D, algo in paths:
    row = []
    for key, xin in inputs.items():
        f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=_lib.C64, algorithm=algo).design(2.4e6)
        dx = DeviceBuffer.from_numpy(xin)
        n_out = f.output_len(n)
        dy = DeviceBuffer.empty(n_out)
        s = f.stream()
        ms = []
        for it in range(7):
            a, b = Event(), Event()
            a.record(s)
            f.process_dev(dx.ptr, n, dy.ptr, n_out)
            b.record(s)
            b.synchronize()
            if it >= 2:
                ms.append(a.elapsed_ms(b))
        row.append(f"{key} {np.median(ms):.3f} ms")
        synchronize()
    print(f"{name:10s} kernel={f.last_kernel()}  " + "  ".join(row), flush=True)
