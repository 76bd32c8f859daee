"""Dump the secondary FIR paths' outputs (VALU direct forms, overlap-save, bf16x3 MFMA, naive) on
seeded finite inputs, for a bitwise comparison of two builds (diagnostic, not a test):
    python tools/experiments/run_with_lib.py A.so tools/diag/fir_paths_dump.py OUT_A.npz
    python tools/diag/fir_paths_dump.py OUT_B.npz
    python tools/diag/fir_bitwise.py --compare OUT_A.npz OUT_B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402

ALG = {"auto": _lib.FIR_AUTO, "direct": _lib.FIR_DIRECT, "os": _lib.FIR_OVERLAP_SAVE}
PATHS = [(0, 0, 127, 1, "auto"), (1, 0, 255, 1, "direct"), (1, 0, 255, 4, "direct"),
         (1, 0, 255, 2, "direct"), (1, 1, 63, 3, "auto"), (1, 0, 255, 4, "os"), (1, 0, 255, 1, "os"),
         (1, 1, 255, 2, "auto"), (1, 0, 255, 8, "auto"), (1, 0, 33, 64, "auto")]
out = {}
for sk, tk, K, D, algo in PATHS:
    rng = np.random.default_rng(K * 10 + D)
    taps = (rng.standard_normal(K) / np.sqrt(K)).astype(np.float32)
    if tk:
        taps = (taps + 1j * rng.standard_normal(K) / np.sqrt(K)).astype(np.complex64)
    n = 300000
    x = rng.standard_normal(n).astype(np.float32)
    if sk:
        x = (x + 1j * rng.standard_normal(n)).astype(np.complex64)
    f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=sk, algorithm=ALG[algo]).design(2.4e6)
    key = f"sk{sk}tk{tk}K{K}D{D}{algo}"
    out[key] = np.concatenate([f.process(x[:n // 3]), f.process(x[n // 3:])])
    out[key + "_kernel"] = np.array([f.last_kernel()])
np.savez(sys.argv[1], **out)
print(sys.argv[1], {k: v.shape for k, v in out.items() if not k.endswith("_kernel")})
