"""Output hashes of the FFT kernels with compile-time frame sizes (gen_fixed_kernel: the
1000-point live spectrum and the 14,400-point transform; fft_tile_kernel: powers of two;
gen_tile_kernel: other smooth sizes)
over full and ragged launches, c64 and rtl_tcp u8 STFT input, c64 and dB output, plain framed fft: run under two builds of the library
(tools/experiments/run_with_lib.py) to show a change left every output bit unchanged.
Diagnostic only."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer, synchronize  # noqa: E402

rng = np.random.default_rng(11)
for n, hop, n_in in ((1000, 500, 1 << 20), (1000, 500, 999_937), (1000, 250, 300_001),
                     (1000, 1700, 500_000), (14400, 7200, 1 << 20), (1024, 512, 1 << 20),
                     (4096, 2048, 1_000_003), (4096, 5000, 600_000), (256, 100, 300_007),
                     (64, 1, 70_001), (1001, 333, 400_003), (3000, 1500, 1 << 20), (1200, 600, 700_001),
                     (6000, 3000, 1 << 20), (600, 250, 300_000), (96, 40, 100_000)):
    for kind in (_lib.C64, _lib.CU8):
        for out in ("complex", "db"):
            s = sdrgpu.fft.Stft(n, hop, input_kind=kind, output=out)
            if kind == _lib.CU8:
                x = rng.integers(0, 256, size=2 * n_in, dtype=np.uint8)
            else:
                x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
            dx = DeviceBuffer(x.nbytes)
            dx.upload(x)
            h = hashlib.sha256()
            for blk in range(2):  # two blocks: the second starts from carried history
                nf = s.output_len(n_in)
                ob = 4 if out == "db" else 8
                dy = DeviceBuffer(max(1, nf * n * ob))
                s.process_dev(dx.ptr, n_in, dy.ptr, nf)
                synchronize()
                h.update(dy.download(nf * n * ob, np.uint8).tobytes())
            print(f"stft n={n} hop={hop} n_in={n_in} in={'u8' if kind == _lib.CU8 else 'c64'} "
                  f"out={out}: {h.hexdigest()[:16]}", flush=True)
for n, frames in ((1000, 4097), (14400, 33), (1024, 1031), (4096, 77), (16, 9999), (1001, 501), (3000, 97),
                  (6000, 41), (600, 777), (96, 5000)):
    x = (rng.standard_normal(n * frames) + 1j * rng.standard_normal(n * frames)).astype(np.complex64)
    for out in ("complex", "db"):
        y = sdrgpu.fft.FftPlan(n, output=out).exec(x.reshape(frames, n))
        print(f"fft n={n} frames={frames} out={out}: {hashlib.sha256(y.tobytes()).hexdigest()[:16]}", flush=True)
for n, frames in ((14400, 37), (14400, 4096)):
    x = rng.standard_normal(n * frames).astype(np.float32)
    for out in ("complex", "db"):
        y = sdrgpu.fft.FftPlan(n, output=out).exec_real(x.reshape(frames, n))
        print(f"rfft n={n} frames={frames} out={out}: {hashlib.sha256(y.tobytes()).hexdigest()[:16]}", flush=True)
