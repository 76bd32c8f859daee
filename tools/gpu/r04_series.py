#!/usr/bin/env python3
"""Per-launch durations of the headline FIR launch under the driver's command shape
(VERDICT r3 item 2): bench.py's own setup, --warmup 5, 20 timed launches, then more
phases in the same process to find what makes the early launches slow.

Phases (each launch bracketed by HIP events on the handle's stream):
  driver   5 untimed warmups + 20 launches (what `bench.py --steps 20 --warmup 5` times)
  long     400 further back-to-back launches
  idle     1 s host sleep (GPU idle), then 40 launches
  memset   1 s sleep, ~200 ms of back-to-back 2 GiB device memsets (HBM busy, no FIR),
           then 40 launches
  fresh    40 launches on a newly allocated input/output pair (first touch of new pages)
Prints one JSON object per phase: per-launch ms, and the mean of the first 5 / last 5."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "unnamed-rust-sdr_amd"))

import bench  # noqa: E402  (synth_iq_pattern: the same data as the headline)


def main():
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer, Event, synchronize
    t_start = time.perf_counter()
    taps = ss.firwin(255, 0.2).astype(np.float32)
    n = 1 << 28
    fir = sdrgpu.filter.Fir(taps, decim=4, sample_kind=_lib.C64, device=0,
                            algorithm=_lib.FIR_AUTO).design(2.4e6)
    stream = fir.stream()
    pat_n = 1 << 22
    pat = bench.synth_iq_pattern(pat_n, seed=1000)

    def make_buffers():
        x = DeviceBuffer.empty(n, np.complex64)
        for off in range(0, n, pat_n):
            x.upload(pat[:min(pat_n, n - off)], offset_bytes=8 * off)
        y = DeviceBuffer.empty(n // 4, np.complex64)
        return x, y

    x, y = make_buffers()
    synchronize(0)
    print(json.dumps({"setup_s": round(time.perf_counter() - t_start, 3)}), flush=True)

    def launches(k, xb, yb):
        ev = [(Event(0), Event(0)) for _ in range(k)]
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            fir.process_dev(xb.ptr, n, yb.ptr, n // 4)
            b.record(stream)
        fir.sync()
        wall = time.perf_counter() - t0
        ms = [a.elapsed_ms(b) for a, b in ev]
        return ms, wall

    def report(name, ms, wall, **kw):
        d = {"phase": name, "launches": len(ms), "wall_ms_per": round(wall / len(ms) * 1e3, 4),
             "mean": round(float(np.mean(ms)), 4), "first5": round(float(np.mean(ms[:5])), 4),
             "last5": round(float(np.mean(ms[-5:])), 4), "min": round(min(ms), 4),
             "ms": [round(v, 4) for v in ms]}
        d.update(kw)
        print(json.dumps(d), flush=True)

    for _ in range(5):
        fir.process_dev(x.ptr, n, y.ptr, n // 4)
    fir.sync()
    ms, wall = launches(20, x, y)
    report("driver", ms, wall)
    ms, wall = launches(400, x, y)
    report("long", ms, wall)
    time.sleep(1.0)
    ms, wall = launches(40, x, y)
    report("idle", ms, wall)
    time.sleep(1.0)
    scratch = DeviceBuffer(2 << 30)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 0.2:
        scratch.fill_zero()
        k += 1
    ms, wall = launches(40, x, y)
    report("memset", ms, wall, memsets=k)
    scratch.free()
    x2, y2 = make_buffers()
    synchronize(0)
    ms, wall = launches(40, x2, y2)
    report("fresh", ms, wall)


if __name__ == "__main__":
    main()
