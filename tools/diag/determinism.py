"""Run-to-run determinism of the MFMA FIR kernels (the packed-f32 fault of DESIGN 3.6 shows as
outputs that change from launch to launch): each shape launched REPS times on the same device
input, every output buffer hashed; prints the number of distinct hashes per shape (1 = every
launch bit-identical).  Diagnostic only."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer, synchronize  # noqa: E402

REPS = int(os.environ.get("REPS", "30"))
rng = np.random.default_rng(9)
taps = (rng.standard_normal(255) / 16).astype(np.float32)
shapes = [("c64 D4 (fir_mxh)", _lib.C64, 4, 1, 1 << 26), ("c64 D2 (fir_mxh)", _lib.C64, 2, 1, 1 << 25),
          ("u8 D4 (fir_mxi)", _lib.CU8, 4, 1, 1 << 26), ("u8 D1 (fir_mxi)", _lib.CU8, 1, 1, 1 << 24),
          ("u8 D8 (fir_mxi)", _lib.CU8, 8, 1, 1 << 25), ("c64 D1 bank 1024 ch (fir_mxh)", _lib.C64, 1, 1024, 1 << 15)]
for name, sk, D, nch, n in shapes:
    if sk == _lib.CU8:
        x = rng.integers(0, 256, size=2 * n * nch, dtype=np.uint8)
    else:
        x = (rng.standard_normal(n * nch) + 1j * rng.standard_normal(n * nch)).astype(np.complex64)
    dx = DeviceBuffer.from_numpy(x)
    if nch > 1:
        f = sdrgpu.filter.FirBank(taps, nch, sample_kind=sk, decim=D)
        n_out = n // D
    else:
        f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=sk).design(2.4e6)
        n_out = f.output_len(n)
    dy = DeviceBuffer.empty(n_out * nch)
    hashes = {}
    for r in range(REPS):
        f.reset()
        if nch > 1:
            f.process_dev(dx.ptr, n, n, dy.ptr, n_out)
        else:
            f.process_dev(dx.ptr, n, dy.ptr, n_out)
        synchronize()
        h = hashlib.sha1(dy.download(n_out * nch, np.complex64).tobytes()).hexdigest()[:12]
        hashes[h] = hashes.get(h, 0) + 1
    print(f"{name:32s} kernel={f.last_kernel()} {REPS} launches, {len(hashes)} distinct outputs {hashes}", flush=True)
