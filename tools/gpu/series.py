#!/usr/bin/env python3
"""Per-launch durations of a FIR launch from the start of a busy period:
bench.py's own setup, then every launch bracketed by HIP events on the handle's stream.

    python tools/gpu/series.py [--kind c64|u8|bank] [--clk]
    python tools/experiments/run_with_lib.py LIB.so tools/gpu/series.py ...   (a variant)

Phases (one JSON line each, per-launch ms in "ms"):
  driver   5 warmups + 20 launches: what `bench.py --steps 20 --warmup 5` runs (warmups
           included in the list, marked by "warmup": 5)
  long     300 further back-to-back launches
  idle     1 s host sleep (GPU idle), then 60 launches
--kind: c64 = configs[1] (the headline), u8 = configs[1] fed from rtl_tcp u8 (bench_configs
c2u8), bank = configs[4]'s 8192-channel D = 1 bank (bench.py's channel-sharded leg), u8dN =
2^26 rtl_tcp u8 samples through the 255-tap FIR at decimation N (1, 2, 8); c64d2 / c64d8 = 2^26
c64 samples at decimation 2 / 8, c64dir4 / c64dir1 / c64os4 = the same forced onto the VALU
direct form (D = 4 / 1) or overlap-save (D = 4); f32d1 = configs[0]'s 127-tap real filter over
2^26 f32 samples.
--clk: the library is tools/experiments/fir_ablate.sh's `clk` variant, which writes per
workgroup (100 MHz ticks, shader-clock ticks) over the launch 4 KiB before its output
pointer; each launch gets its own output offset so the records survive, and every phase
line carries the per-launch mean shader clock in MHz ("mhz")."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "unnamed-rust-sdr_amd"))

import bench  # noqa: E402  (synth_iq_pattern: the same data as the headline)

GUARD = 1024  # c64 elements (8 KiB) of output offset per launch under --clk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="c64", choices=["c64", "u8", "bank", "u8d1", "u8d2", "u8d8", "c64d2",
                                                      "c64d8", "c64dir4", "c64dir1", "c64os4", "f32d1"])
    ap.add_argument("--clk", action="store_true")
    ap.add_argument("--long", type=int, default=300)
    args = ap.parse_args()
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer, Event, synchronize
    t_start = time.perf_counter()
    taps = ss.firwin(255, 0.2).astype(np.float32)
    nlaunch = 25 + args.long + 60
    guard = GUARD if args.clk else 0
    if args.kind == "bank":
        nch, n = 8192, 1 << 16
        f = sdrgpu.filter.FirBank(taps, nch, sample_kind=_lib.C64)
        x = DeviceBuffer.empty(nch * n, np.complex64)
        pat = bench.synth_iq_pattern(1 << 22, seed=4000)
        for off in range(0, nch * n, pat.size):
            x.upload(pat[:min(pat.size, nch * n - off)], offset_bytes=8 * off)
        out_n = nch * n
        y = DeviceBuffer.empty(out_n + guard * (nlaunch + 1), np.complex64)

        def launch(i):
            f.process_dev(x.ptr, n, n, y.ptr + 8 * guard * (i + 1), n)
    elif args.kind in ("c64d2", "c64d8", "c64dir4", "c64dir1", "c64os4"):
        # 2^26 c64 samples: decimation 2 / 8 (AUTO), or D = 4 / 1 forced onto the VALU direct
        # form / D = 4 onto overlap-save (the secondary paths)
        n = 1 << 26
        dec = {"c64d2": 2, "c64d8": 8, "c64dir4": 4, "c64dir1": 1, "c64os4": 4}[args.kind]
        algo = {"c64dir4": _lib.FIR_DIRECT, "c64dir1": _lib.FIR_DIRECT,
                "c64os4": _lib.FIR_OVERLAP_SAVE}.get(args.kind, _lib.FIR_AUTO)
        f = sdrgpu.filter.Fir(taps, decim=dec, sample_kind=_lib.C64, algorithm=algo).design(2.4e6)
        pat = bench.synth_iq_pattern(1 << 22, seed=1000)
        x = DeviceBuffer.empty(n, np.complex64)
        for off in range(0, n, pat.size):
            x.upload(pat[:min(pat.size, n - off)], offset_bytes=8 * off)
        out_n = n // dec
        y = DeviceBuffer.empty(out_n + guard * (nlaunch + 1), np.complex64)

        def launch(i):
            f.process_dev(x.ptr, n, y.ptr + 8 * guard * (i + 1), out_n)
    elif args.kind == "f32d1":  # configs[0]'s filter (127 real taps) over 2^26 f32 samples
        n = 1 << 26
        f = sdrgpu.filter.Fir(ss.firwin(127, 0.2).astype(np.float32), decim=1,
                              sample_kind=_lib.F32).design(2.4e6)
        x = DeviceBuffer.empty(n, np.float32)
        pat = np.random.default_rng(22).standard_normal(1 << 22).astype(np.float32)
        for off in range(0, n, pat.size):
            x.upload(pat[:min(pat.size, n - off)], offset_bytes=4 * off)
        out_n = n
        y = DeviceBuffer.empty(out_n + guard * (nlaunch + 1), np.float32)

        def launch(i):
            f.process_dev(x.ptr, n, y.ptr + 4 * guard * (i + 1), out_n)
    elif args.kind.startswith("u8d"):  # u8 stream, decimation 1 / 2 / 8: 2 B in + 8/D B out per sample
        n = 1 << 26
        dec = int(args.kind[3:])
        f = sdrgpu.filter.Fir(taps, decim=dec, sample_kind=_lib.CU8).design(2.4e6)
        pat = np.random.default_rng(21).integers(0, 256, size=2 * (1 << 22), dtype=np.uint8)
        x = DeviceBuffer.empty(2 * n, np.uint8)
        for off in range(0, 2 * n, pat.size):
            x.upload(pat[:min(pat.size, 2 * n - off)], offset_bytes=off)
        out_n = n // dec
        y = DeviceBuffer.empty(out_n + guard * (nlaunch + 1), np.complex64)

        def launch(i):
            f.process_dev(x.ptr, n, y.ptr + 8 * guard * (i + 1), out_n)
    else:
        n = 1 << 28
        kind = _lib.C64 if args.kind == "c64" else _lib.CU8
        f = sdrgpu.filter.Fir(taps, decim=4, sample_kind=kind).design(2.4e6)
        if args.kind == "c64":
            pat = bench.synth_iq_pattern(1 << 22, seed=1000)
            x = DeviceBuffer.empty(n, np.complex64)
            for off in range(0, n, pat.size):
                x.upload(pat[:min(pat.size, n - off)], offset_bytes=8 * off)
        else:
            pat = np.random.default_rng(21).integers(0, 256, size=2 * (1 << 22), dtype=np.uint8)
            x = DeviceBuffer.empty(2 * n, np.uint8)
            for off in range(0, 2 * n, pat.size):
                x.upload(pat[:min(pat.size, 2 * n - off)], offset_bytes=off)
        out_n = n // 4
        y = DeviceBuffer.empty(out_n + guard * (nlaunch + 1), np.complex64)

        def launch(i):
            f.process_dev(x.ptr, n, y.ptr + 8 * guard * (i + 1), out_n)
    stream = f.stream()
    synchronize(0)
    print(json.dumps({"kind": args.kind, "setup_s": round(time.perf_counter() - t_start, 3)}), flush=True)
    counter = [0]

    def launches(k):
        ev = [(Event(0), Event(0)) for _ in range(k)]
        first = counter[0]
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            launch(counter[0])
            counter[0] += 1
            b.record(stream)
        f.sync()
        wall = time.perf_counter() - t0
        ms = [a.elapsed_ms(b) for a, b in ev]
        mhz = None
        if args.clk:
            mhz = []
            for i in range(first, first + k):
                rec = y.download(512, dtype=np.uint64, offset_bytes=8 * guard * (i + 1) - 4096)
                rt, ck = rec[0::2].astype(np.float64), rec[1::2].astype(np.float64)
                ok = rt > 0
                mhz.append(round(float(ck[ok].sum() / rt[ok].sum() * 100.0), 1) if ok.any() else None)
        return ms, wall, mhz

    def report(name, ms, wall, mhz, **kw):
        d = {"phase": name, "kind": args.kind, "launches": len(ms),
             "wall_ms_per": round(wall / len(ms) * 1e3, 4), "mean": round(float(np.mean(ms)), 4),
             "min": round(min(ms), 4), "ms": [round(v, 4) for v in ms]}
        if mhz is not None:
            d["mhz"] = mhz
        d.update(kw)
        print(json.dumps(d), flush=True)

    ms, wall, mhz = launches(25)
    report("driver", ms, wall, mhz, warmup=5, timed_mean=round(float(np.mean(ms[5:])), 4))
    ms, wall, mhz = launches(args.long)
    report("long", ms, wall, mhz)
    time.sleep(1.0)
    ms, wall, mhz = launches(60)
    report("idle", ms, wall, mhz)


if __name__ == "__main__":
    main()
