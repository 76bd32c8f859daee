"""examples/live.rs spectrum shape (1000-point STFT, hop 500) over 2^26 c64 samples: kernel time
with c64 output vs the fused dB output vs u8 input + dB, HIP events on the handle's stream,
median of 10 after 3 warmups.  Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer, Event  # noqa: E402

n_in = 1 << 26
rng = np.random.default_rng(3)
x = (rng.standard_normal(1 << 22) + 1j * rng.standard_normal(1 << 22)).astype(np.complex64)
xu = rng.integers(0, 256, size=2 << 22, dtype=np.uint8)
for n, hop in ((1000, 500), (1024, 512), (4096, 2048), (1200, 600), (3000, 1500), (6000, 3000)):
    for out, kind in (("complex", _lib.C64), ("db", _lib.C64), ("db", _lib.CU8)):
        s = sdrgpu.fft.Stft(n, hop, input_kind=kind, output=out)
        eb = 2 if kind == _lib.CU8 else 8
        dx = DeviceBuffer(n_in * eb)
        pat = xu if kind == _lib.CU8 else x
        for off in range(0, n_in * eb, pat.nbytes):
            dx.upload(pat[:min(pat.size, (n_in * eb - off) // pat.itemsize)], offset_bytes=off)
        nf = s.output_len(n_in)
        ob = 4 if out == "db" else 8
        dy = DeviceBuffer(nf * n * ob)
        st = s.stream()
        ms = []
        for it in range(13):
            s.reset()
            a, b = Event(), Event()
            a.record(st)
            s.process_dev(dx.ptr, n_in, dy.ptr, nf)
            b.record(st)
            b.synchronize()
            if it >= 3:
                ms.append(a.elapsed_ms(b))
        byt = n_in * eb + nf * n * ob
        t = float(np.median(ms))
        print(f"n={n} hop={hop} in={'u8' if kind == _lib.CU8 else 'c64'} out={out:7s} {t:.4f} ms  "
              f"{byt / t / 1e9:.0f} GB/s = {byt / t / 8e9:.3f} of 8 TB/s", flush=True)
# examples/fft.rs: 14,400-point rfft over 4096 real frames (packed half-length kernel)
for out in ("complex", "db"):
    p = sdrgpu.fft.FftPlan(14400, output=out)
    xr = rng.standard_normal(14400 * 4096).astype(np.float32)
    dx = DeviceBuffer(xr.nbytes)
    dx.upload(xr)
    ob = 4 if out == "db" else 8
    dy = DeviceBuffer(4096 * 7200 * ob)
    st = p.stream()
    ms = []
    for it in range(13):
        a, b = Event(), Event()
        a.record(st)
        p.exec_real_dev(dx.ptr, dy.ptr, 4096)
        b.record(st)
        b.synchronize()
        if it >= 3:
            ms.append(a.elapsed_ms(b))
    t = float(np.median(ms))
    byt = xr.nbytes + 4096 * 7200 * ob
    print(f"n=14400 rfft x4096 out={out:7s} {t:.4f} ms  {byt / t / 8e9:.3f} of 8 TB/s", flush=True)
