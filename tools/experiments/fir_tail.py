"""Tail census of the headline FIR launch (run through run_with_lib.py with fir_ablate.sh's
wgtime library, which writes each workgroup's start/end s_memrealtime into out[0..511]):
how long after the first workgroup finishes does the last one finish?"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer, Event, synchronize  # noqa: E402

n = 1 << 28
taps = ss.firwin(255, 0.2).astype(np.float32)
fir = sdrgpu.filter.Fir(taps, decim=4, sample_kind=_lib.C64, device=0).design(2.4e6)
pat = bench.synth_iq_pattern(1 << 22, seed=1000)
x = DeviceBuffer.empty(n, np.complex64, device=0)
for off in range(0, n, 1 << 22):
    x.upload(pat, offset_bytes=8 * off)
y = DeviceBuffer.empty(n // 4, np.complex64, device=0)
e0, e1 = Event(0), Event(0)
REPS = int(os.environ.get('TAIL_REPS', '6'))
summ = []
for rep in range(REPS):
    e0.record(fir.stream())
    fir.process_dev(x.ptr, n, y.ptr, n // 4)
    e1.record(fir.stream())
    fir.sync()
    ev_us = e0.elapsed_ms(e1) * 1e3
    synchronize(0)
    t = np.frombuffer(y.download(512).tobytes(), dtype=np.uint64)[:512].reshape(256, 2)
    xcc = (t[:, 0] >> np.uint64(56)).astype(int)
    s = (t[:, 0] & np.uint64((1 << 56) - 1)).astype(np.int64)
    e = t[:, 1].astype(np.int64)
    s0 = s.min()
    ends = np.sort((e - s0) / 100.0)
    byx = collections.defaultdict(list)
    for xi, ei in zip(xcc, (e - s0) / 100.0):
        byx[xi].append(ei)
    summ.append((ev_us, ends[-1], float(np.mean(ends)), ends[0]))
    if rep >= REPS - 4 or rep < 2:
      print(f"rep {rep}: event {ev_us:.1f} us, span {ends[-1]:.1f} us, start spread {(s.max() - s0) / 100.0:.1f} us, end "
          f"min/p10/p50/p90/max {ends[0]:.1f}/{ends[25]:.1f}/{ends[128]:.1f}/{ends[230]:.1f}/{ends[-1]:.1f} us; "
          "per-XCD mean end " + " ".join(f"{k}:{np.mean(v):.1f}" for k, v in sorted(byx.items())))
a = np.array(summ[len(summ) // 2:])
print(f"last {len(a)} reps: event {a[:, 0].mean():.1f} us, last end {a[:, 1].mean():.1f}, mean end {a[:, 2].mean():.1f}, "
      f"first end {a[:, 3].mean():.1f} us -> a balanced split would save {(a[:, 1] - a[:, 2]).mean():.1f} us "
      f"({100 * (a[:, 1] - a[:, 2]).mean() / a[:, 0].mean():.1f} %)")
