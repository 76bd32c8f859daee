"""Time-parallel biquad vs the serial pass (round 5): a few long streams through BiquadD
designs of src/main.rs (the PLL's lock filter at 1.8 Msps, the de-emphasis Lr and the pilot
filter at 144 kHz); device-resident blocks, HIP events on the handle's stream, outputs of the
two plans compared bit for bit.  python tools/diag/bq_tp_bench.py > out.jsonl"""
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import sdrgpu  # noqa: E402
from sdrgpu.device import DeviceBuffer, Event  # noqa: E402

f = sdrgpu.filter
CASES = [("lock LowPass(20 kHz, 0.7) @ 1.8 Msps", f.BiquadD.LowPass(20000.0, 0.7), 1.8e6),
         ("de-emphasis Lr(1/75 us) @ 144 kHz", f.BiquadD.Lr(1.0 / 75e-6), 144000.0),
         ("pilot loop LowPass(200 Hz, 0.7) @ 144 kHz", f.BiquadD.LowPass(200.0, 0.7), 144000.0),
         ("pilot LowPass(20 Hz, 0.7) @ 144 kHz", f.BiquadD.LowPass(20.0, 0.7), 144000.0)]
n = 1 << 22
rng = np.random.default_rng(5)
for name, d, rate in CASES:
    for sk in (0, 1):
        for nch in (1, 2, 64):
            dt = np.complex64 if sk else np.float32
            x = rng.standard_normal((nch, n)).astype(np.float32)
            if sk:
                x = (x + 1j * rng.standard_normal((nch, n)).astype(np.float32)).astype(dt)
            dx = DeviceBuffer.from_numpy(np.ascontiguousarray(x))
            res = {"case": name, "kind": "c64" if sk else "f32", "nch": nch, "n": n}
            outs = {}
            for plan in ("serial", "auto"):
                bq = d.design(rate, sample_kind=sk, nch=nch)
                if plan == "serial":
                    bq.set_time_parallel(-1)
                dy = DeviceBuffer.empty(nch * n, dt)
                bq.process_dev(dx.ptr, n, n, dy.ptr, n)  # warm (state then reset)
                bq.sync()
                bq.reset()
                e0, e1 = Event(), Event()
                s = bq.stream()
                e0.record(s)
                bq.process_dev(dx.ptr, n, n, dy.ptr, n)
                e1.record(s)
                e1.synchronize()
                ms = e0.elapsed_ms(e1)
                segs, rec = bq.last_time_parallel()
                outs[plan] = dy.download(nch * n, dt)
                res[plan] = {"ms": round(ms, 4), "ns_per_sample_of_batch": round(ms * 1e6 / (nch * n), 3),
                             "segments": segs, "recomputed": rec, "plan": bq.time_parallel_plan(n)}
            res["bit_identical"] = bool(np.array_equal(outs["serial"].view(np.uint32), outs["auto"].view(np.uint32)))
            res["speedup"] = round(res["serial"]["ms"] / res["auto"]["ms"], 1)
            print(json.dumps(res), flush=True)
