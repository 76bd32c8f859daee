"""Time-parallel PLL on ONE stream in main.rs's 0.1 s blocks (the FM receiver's discriminator:
rtl_tcp u8 I/Q at 1.8 Msps, 180000 samples per block): PLL time per block and segments re-run,
per (segment, warm-up) plan, outputs compared with the serial plan bit for bit.
python tools/diag/pll_tp_single.py seg:warm ...   (seg 0 = the automatic plan)"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import bench_configs as bc  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu import fm  # noqa: E402
from sdrgpu.device import DeviceBuffer, Event  # noqa: E402

blk, nblk = 180000, 20
raw = bc.fm_stereo_u8(blk * nblk)
dx = DeviceBuffer.from_numpy(raw)
plans = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(0, 0)]
ref = None
for seg, warm in [(-1, 0)] + plans:
    pll = fm.discriminator_design().design(fm.RATE, nch=1)
    pll.set_input_kind(sdrgpu._lib.CU8)
    pll.set_time_parallel(seg, warm)
    out = DeviceBuffer.empty(blk * nblk, np.float32)
    lk = DeviceBuffer.empty(blk * nblk, np.uint8)
    s = pll.stream()
    ms, rec = [], 0
    for b in range(nblk):
        e0, e1 = Event(), Event()
        e0.record(s)
        pll.process_dev(dx.ptr + 2 * blk * b, blk, blk, out.ptr + 4 * blk * b, lk.ptr + blk * b, blk)
        e1.record(s)
        e1.synchronize()
        ms.append(e0.elapsed_ms(e1))
        rec += pll.last_time_parallel()[1]
    o = out.download(blk * nblk, np.float32)
    same = None
    if ref is None:
        ref = o
    else:
        same = bool(np.array_equal(o.view(np.uint32), ref.view(np.uint32)))
    print(f"seg {seg:6d} warm {warm:6d}: plan {pll.time_parallel_plan(blk)}  {np.mean(ms[2:]):7.3f} ms per block "
          f"(min {np.min(ms[2:]):.3f}), re-run {rec}, identical to serial: {same}", flush=True)
