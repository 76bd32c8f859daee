#!/usr/bin/env python3
"""bench_configs.py -- measurements for the other BASELINE.json configs.

bench.py is the driver's headline line (configs[1]); this script measures configs[2..4]
with the same rules (inputs resident in HBM, HIP-event-timed kernels on the handle's
stream, algorithmic bytes per input sample, a bounded CPU-baseline sample), one JSON line
per config:

  c1  127-tap real FIR over 2^20 f32 (configs[0], the reference CPU path): oracle on 1
      host core, the same block on the GPU beside it
  c3  64k-point STFT, 50 % overlap, 2^28 c64 samples      24 B / input sample, HBM roof
  c4  255-tap matched filter (FIR bank) + PLL FM demod,    12 B / input sample (+1 lock);
      1024 channels x 2^20 c64                              PLL = loop-carried latency
  c5  255-tap FIR bank, channels sharded across GPUs,      16 B / input sample, HBM roof
      8192 channels x 2^16 c64 (1024 per GPU at 8 GPUs)
  c2u8  configs[1] fed from rtl_tcp u8 IQ:    2 B in + 2 B out / sample
      (v-128)/128 fused into the FIR load, 2^28 samples

Multi-GPU (c5): `python -m torch.distributed.run --nproc-per-node N bench_configs.py
--config c5`; each rank filters its resident channel shard (weak: 8192/N channels per rank
... see --c5-weak), and RCCL scatter (root -> ranks) / gather (ranks -> root) of the
channel blocks is timed separately ("fan-out/gather only", north_star).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "unnamed-rust-sdr_amd"))
sys.path.insert(0, ROOT)

HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="all", choices=["c1", "c3", "c4", "c5", "c2u8", "c2host", "c2pinned", "src", "ex", "fm", "all"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--c3-log2n", type=int, default=28)
    ap.add_argument("--c4-log2n", type=int, default=20)
    ap.add_argument("--c4-nch", type=int, default=1024)
    ap.add_argument("--c5-nch", type=int, default=8192)
    ap.add_argument("--c5-log2n", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--fm-seconds", type=float, default=10.0, help="seconds of air through the fm chain")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="timing-only ablation builds: skip the c3 / c5 spot checks")
    ap.add_argument("--gpus", type=int, default=1,
                    help="c5 only: run as this many ranks (self-launched, one process per GPU)")
    return ap.parse_args()


def cplx_pattern(n, seed):
    r = np.random.default_rng(seed)
    return ((r.standard_normal(n, dtype=np.float32) + 1j * r.standard_normal(n, dtype=np.float32))
            * 0.3).astype(np.complex64)


def fill(buf, n, seed, pat_n=1 << 22):
    pat = cplx_pattern(min(n, pat_n), seed)
    for off in range(0, n, len(pat)):
        buf.upload(pat[:min(len(pat), n - off)], offset_bytes=8 * off)


def time_events(step, stream, steps, warmup, sync):
    from sdrgpu.device import Event
    for _ in range(warmup):
        step()
    sync()
    ev = [(Event(), Event()) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    sync()
    wall = (time.perf_counter() - t0) / steps
    return wall, float(np.mean([a.elapsed_ms(b) for a, b in ev]))


def roof(bytes_per_unit, units, ms):
    gbs = bytes_per_unit * units / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_GBS, 4), "kernel_ms": round(ms, 4)}


# ------------------------------------------------------------------------------ c1
def bench_c1(args):
    """configs[0]: the reference's CPU path -- a 127-tap real lowpass FIR over 2^20 f32
    samples (examples/filter.rs's signal.filter(...) shape with FIR taps) -- timed as the
    oracle restatement on one host core; the same block on the GPU beside it."""
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu.device import DeviceBuffer, synchronize
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from bench import host_info
    n = 1 << 20
    taps = ss.firwin(127, 0.2).astype(np.float32)
    x = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    o = pyoracle.Fir(taps, 1, sample_kind=0)
    t0, done = time.perf_counter(), 0
    while True:
        ref = o.process(x)
        done += n
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    fir = sdrgpu.filter.Fir(taps, sample_kind=sdrgpu.F32).design(44100.0)
    dx = DeviceBuffer.from_numpy(x)
    dy = DeviceBuffer.empty(n, np.float32)

    def step():
        assert fir.process_dev(dx.ptr, n, dy.ptr, n) == n

    wall, ms = time_events(step, fir.stream(), args.steps, args.warmup,
                           lambda: (fir.sync(), synchronize()))
    # parity of the last GPU block: its FIR history is the block's own tail (steady state)
    y = dy.download(dtype=np.float32)
    prev = o.process(x)  # the oracle continues its own stream over the same block
    err = float(np.abs(y - prev).max() / np.sqrt(np.mean(prev.astype(np.float64) ** 2)))
    assert err <= 1e-5, err
    return {"config": "c1: 127-tap real FIR (firwin 0.2), 2^20 f32 samples -- configs[0], "
                      "the reference CPU path",
            "metric": "Msamples/s (f32 input)",
            "cpu_baseline": {"value": round(done / el / 1e6, 2), "unit": "Msamples/s", "cores": 1,
                             "kind": "port", "host": host_info(),
                             "sample": f"{done // n} passes of 2^20 f32 samples through the "
                                       f"oracle Fir (127 taps), {el:.1f} s on 1 host core"},
            "gpu": {"value": round(n / (ms * 1e-3) / 1e6, 1), "kernel_ms": round(ms, 4),
                    "algorithm": fir.last_algorithm(), "wall_ms_per_step": round(wall * 1e3, 3),
                    "parity_max_over_rms": err,
                    "roofline": roof(8, n, ms)}}


# ------------------------------------------------------------------------------ c3
def bench_c3(args):
    import sdrgpu
    from sdrgpu.device import DeviceBuffer, synchronize
    N, hop = 65536, 32768
    n = 1 << args.c3_log2n
    st = sdrgpu.fft.Stft(N, hop)
    x = DeviceBuffer.empty(n)
    fill(x, n, 3)
    nf = st.output_len(n)
    y = DeviceBuffer.empty(nf * N)

    def step():
        st.reset()
        assert st.process_dev(x.ptr, n, y.ptr, nf) == nf

    wall, ms = time_events(step, st.stream(), args.steps, args.warmup, lambda: (st.sync(), synchronize()))
    # spot check of the timed outputs (the last step's): frames at the first scratch-batch
    # boundaries (both streams of the multi-batch schedule) and the last frame, each against
    # the oracle FFT of its own span of the tiled input pattern
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pat = cplx_pattern(min(n, 1 << 22), 3)
    worst = 0.0
    for j in (0, 255, 256, nf - 1):
        g = np.arange((j + 1) * hop - N, (j + 1) * hop)
        span = np.where(g >= 0, pat[np.maximum(g, 0) % pat.size], 0).astype(np.complex64)
        ref = pyoracle.fft_frame(span).astype(np.complex128)
        got = y.download(N, offset_bytes=8 * N * j)
        worst = max(worst, float(np.abs(got - ref).max() / np.sqrt(np.mean(np.abs(ref) ** 2))))
    assert worst <= 1e-5 or args.no_check, worst
    res = {"config": "c3: 64k-point STFT, 50% overlap, fftshift + 1/sqrt(N), 2^28 c64 samples",
           "metric": "complex Msamples/s (input)", "value": round(n / (ms * 1e-3) / 1e6, 1),
           "frames": nf, "roofline": roof(24, n, ms), "wall_ms_per_step": round(wall * 1e3, 3),
           "spot_check_max_over_rms": worst}
    if not args.no_cpu_baseline:
        xf = cplx_pattern(N, 7)
        t0, done = time.perf_counter(), 0
        while time.perf_counter() - t0 < args.cpu_seconds:
            np.fft.fftshift(np.fft.fft(xf)) / np.float32(np.sqrt(N))
            done += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(done * hop / el / 1e6, 2), "unit": "complex Msamples/s",
                               "cores": 1, "kind": "proxy",
                               "sample": f"{done} NumPy pocketfft 64k frames (proxy for rustfft 3.0), {el:.1f} s"}
    return res


# ------------------------------------------------------------------------------ ex
def bench_ex(args):
    """The reference examples' FFT shapes at throughput scale (not BASELINE configs): the
    live spectrum of examples/live.rs (1000-point frames of rtl_tcp-rate IQ, shown in dB by
    ComplexSeries::plot) as an STFT with hop 500 and the fused dB output, and the
    14,400-point rfft of examples/fft.rs (take(0.1) at 144 kHz) batched over 4096 frames --
    both through the any-N (mixed-radix 2/3/5) kernels."""
    import sdrgpu
    from sdrgpu.device import DeviceBuffer, synchronize
    out = []
    n = 1 << 26
    st = sdrgpu.fft.Stft(1000, 500, output="db")
    x = DeviceBuffer.empty(n)
    fill(x, n, 21)
    nf = st.output_len(n)
    y = DeviceBuffer.empty(nf * 1000 // 2 + 1)  # f32 dB values: half the c64 bytes

    def step():
        st.reset()
        assert st.process_dev(x.ptr, n, y.ptr, nf) == nf

    wall, ms = time_events(step, st.stream(), args.steps, args.warmup, lambda: (st.sync(), synchronize()))
    out.append({"config": "ex_live: examples/live.rs spectrum shape -- 1000-point STFT, hop 500, "
                          "fused 20*log10|X| (f32) output, 2^26 c64 samples",
                "metric": "complex Msamples/s (input)", "value": round(n / (ms * 1e-3) / 1e6, 1),
                "frames": nf, "roofline": roof(8 + 2 * 4, n, ms), "wall_ms_per_step": round(wall * 1e3, 3)})
    N, count = 14400, 4096
    p = sdrgpu.fft.FftPlan(N)
    xr = DeviceBuffer.empty(N * count // 2)  # f32 frames (c64-sized buffer units)
    fill(xr, N * count // 2, 22)
    yr = DeviceBuffer.empty((N - N // 2) * count)

    def step2():
        p.exec_real_dev(xr.ptr, yr.ptr, count)

    wall, ms = time_events(step2, p.stream(), args.steps, args.warmup, lambda: (p.sync(), synchronize()))
    out.append({"config": "ex_rfft: examples/fft.rs rfft shape -- 14400-point rfft (f32 in, 7200 "
                          "c64 bins out) x 4096 frames",
                "metric": "real Msamples/s (input)", "value": round(N * count / (ms * 1e-3) / 1e6, 1),
                "roofline": roof(4 + 4, N * count, ms), "wall_ms_per_step": round(wall * 1e3, 3)})
    return out


# ------------------------------------------------------------------------------ c2u8
def bench_c2u8(args):
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu.device import DeviceBuffer, synchronize
    n = 1 << 28
    taps = ss.firwin(255, 0.2).astype(np.float32)
    fir = sdrgpu.filter.Fir(taps, decim=4, sample_kind=sdrgpu.CU8).design(2.4e6)
    pat = np.random.default_rng(21).integers(0, 256, size=2 * (1 << 22), dtype=np.uint8)
    x = DeviceBuffer.empty(2 * n, np.uint8)
    for off in range(0, 2 * n, pat.size):
        x.upload(pat[:min(pat.size, 2 * n - off)], offset_bytes=off)
    n_out = n // 4
    y = DeviceBuffer.empty(n_out, np.complex64)

    def step():
        assert fir.process_dev(x.ptr, n, y.ptr, n_out) == n_out

    wall, ms = time_events(step, fir.stream(), args.steps, args.warmup,
                           lambda: (fir.sync(), synchronize()))
    # spot check of the timed outputs (the last step's): the first 4096 and the 4096 outputs
    # from 2^25 on (the input pattern repeats every 2^22 samples, so that window's input is
    # the pattern again), against the oracle fed the converted u8 codes.  The handle streams:
    # the last step's history is the end of the step before it (the pattern's tail again).
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    worst = 0.0
    for m0 in (0, 1 << 25):
        j0 = 4 * m0  # a multiple of the pattern period: the window starts the pattern again
        first_call = j0 == 0 and args.steps + args.warmup == 1
        hist = np.full(2 * 256, 128, np.uint8) if first_call else pat[-2 * 256:]
        xin = np.concatenate([hist, pat[:2 * 4 * 4096]])
        ref = pyoracle.Fir(taps, 4, sample_kind=1).process(pyoracle.u8_to_c64(xin))[64:64 + 4096]
        got = y.download(4096, offset_bytes=8 * m0)
        worst = max(worst, float(np.abs(got - ref).max() / np.sqrt(np.mean(np.abs(ref) ** 2))))
    assert worst <= 1e-5 or args.no_check, worst
    return {"config": "c2u8: configs[1] (255-tap FIR, decim 4) fed from rtl_tcp u8 IQ, "
                      "(v-128)/128 fused into the load, 2^28 samples",
            "metric": "complex Msamples/s (input)", "value": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": roof(2 + 8 / 4, n, ms), "wall_ms_per_step": round(wall * 1e3, 3),
            "kernel": "fir_mxi_kernel<5> (int8 MFMA)", "spot_check_max_over_rms": worst}


# ------------------------------------------------------------------------------ c2host
def bench_c2host(args):
    """configs[1] through the HOST-pointer entry point (sdrgpu_fir_process: pageable numpy
    buffers, H2D + kernel + D2H on the handle's stream): the PCIe-inclusive rate."""
    import scipy.signal as ss
    import sdrgpu
    n = 1 << 26
    taps = ss.firwin(255, 0.2).astype(np.float32)
    fir = sdrgpu.filter.Fir(taps, decim=4, sample_kind=sdrgpu.C64).design(2.4e6)
    x = cplx_pattern(n, 5)
    fir.process(x)  # warm-up (staging buffers)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = fir.process(x)
    el = (time.perf_counter() - t0) / args.steps
    assert y.size == n // 4
    return {"config": "c2host: configs[1] via sdrgpu_fir_process (pageable host buffers, "
                      "H2D + FIR + D2H), 2^26 samples per call",
            "metric": "complex Msamples/s (input, PCIe-inclusive)", "value": round(n / el / 1e6, 1),
            "wall_ms_per_call": round(el * 1e3, 3),
            "host_bytes_per_s": round(10 * n / el / 1e9, 2)}


# ------------------------------------------------------------------------------ c2pinned
def bench_c2pinned(args):
    """configs[1] streamed from HOST memory the way the Block adapter would
    (src/signal/adapters/block.rs:105-207): two pinned input/output block pairs, each block
    enqueued with sdrgpu_fir_process_async (H2D + FIR + D2H, no wait) so block i+1's
    transfer queues behind block i's; C64 samples and rtl_tcp u8 bytes."""
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu.device import PinnedBuffer
    n = 1 << 24  # samples per block
    nblocks = 16
    taps = ss.firwin(255, 0.2).astype(np.float32)
    res = {"config": "c2pinned: configs[1] from pinned host blocks of 2^24 samples, async "
                     "H2D + FIR + D2H, 2 blocks in flight (PCIe-inclusive)"}
    for kind, name, ib in ((sdrgpu.C64, "c64", 8), (sdrgpu.CU8, "u8", 2)):
        fir = sdrgpu.filter.Fir(taps, decim=4, sample_kind=kind).design(2.4e6)
        ins = [PinnedBuffer(n * ib, np.uint8) for _ in range(2)]
        outs = [PinnedBuffer(n // 4, np.complex64) for _ in range(2)]
        pat = np.random.default_rng(6).integers(0, 256, size=n * ib, dtype=np.uint8)
        for b in ins:
            b.array[:] = pat
        for i in range(2):  # warm-up (staging buffers)
            fir.process_async(ins[i].ptr, n, outs[i].ptr, n // 4)
        fir.sync()
        t0 = time.perf_counter()
        for i in range(nblocks):
            assert fir.process_async(ins[i & 1].ptr, n, outs[i & 1].ptr, n // 4) == n // 4
        fir.sync()
        el = (time.perf_counter() - t0) / nblocks
        res[name] = {"value": round(n / el / 1e6, 1), "unit": "complex Msamples/s (input)",
                     "ms_per_block": round(el * 1e3, 3),
                     "host_bytes_per_s_GB": round((ib + 2) * n / el / 1e9, 2)}
        for b in ins + outs:
            b.free()
    return res


def spot_check(pyoracle, taps, x, y, ch, n, m=4096):
    """Channel `ch` of a D = 1 bank whose every step filtered the same resident block:
    the state entering a step is the block's own last K-1 samples (the steady state)."""
    K = len(taps)
    tail = x.download(K - 1, offset_bytes=8 * (ch * n + n - (K - 1)))
    xin = x.download(m, offset_bytes=8 * ch * n)
    ref = pyoracle.Fir(taps, 1, sample_kind=1).process(np.concatenate([tail, xin]))[K - 1:]
    got = y.download(m, offset_bytes=8 * ch * n)
    return float(np.abs(got.astype(np.complex128) - ref).max() /
                 np.sqrt(np.mean(np.abs(ref.astype(np.complex128)) ** 2)))


# ------------------------------------------------------------------------------ c4
def bench_c4(args):
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu.device import DeviceBuffer, synchronize
    f = sdrgpu.filter
    nch, n = args.c4_nch, 1 << args.c4_log2n
    rate = 1.8e6
    taps = ss.firwin(255, 0.2).astype(np.float32)
    bank = f.FirBank(taps, nch, sample_kind=sdrgpu.C64)
    pll = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                      f.BiquadD.LowPass(20000.0, 0.7)).design(rate, nch=nch)
    pll.set_stream(bank.stream())
    x = DeviceBuffer.empty(nch * n)
    fill(x, nch * n, 4)
    mf = DeviceBuffer.empty(nch * n)
    out = DeviceBuffer.empty(nch * n, np.float32)
    lk = DeviceBuffer.empty(nch * n, np.uint8)

    def step():
        bank.process_dev(x.ptr, n, n, mf.ptr, n)
        pll.process_dev(mf.ptr, n, n, out.ptr, lk.ptr, n)

    wall, ms = time_events(step, bank.stream(), args.steps, args.warmup, lambda: (bank.sync(), synchronize()))
    # split: matched filter alone
    _, ms_fir = time_events(lambda: bank.process_dev(x.ptr, n, n, mf.ptr, n), bank.stream(),
                            args.steps, 0, lambda: (bank.sync(), synchronize()))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    units = nch * n
    fir_check = spot_check(pyoracle, taps, x, mf, nch // 3, n)
    assert fir_check <= 1e-5, fir_check
    # PLL spot check of the timed path (time-parallel segments at this shape): a fresh handle
    # of the same design and plan over the whole resident matched-filter output; 4 channels'
    # outputs and lock flags array_equal to the oracle PLL (src/filter/pll.rs:70-85), which
    # is the serial recurrence
    pll_v = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                        f.BiquadD.LowPass(20000.0, 0.7)).design(rate, nch=nch)
    pll_v.set_stream(bank.stream())
    pll_v.set_phase_timing(True)
    plan = pll_v.time_parallel_plan(n)
    pll_v.process_dev(mf.ptr, n, n, out.ptr, lk.ptr, n)
    bank.sync()
    tp_segments, tp_recomputed = pll_v.last_time_parallel()
    ph = pll_v.last_phase_ms()  # pass 1 / re-run pass / walk of that block (events on its stream)
    p = pyoracle.pll_params(0.0, 0.035, rate, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
    chans = sorted({0, nch // 3, nch // 2 + 1, nch - 1})
    mfs = np.stack([mf.download(n, offset_bytes=8 * c * n) for c in chans])
    ref_out, ref_lk = pyoracle.pll_batch(p, mfs, nthreads=len(chans))
    got_out = np.stack([out.download(n, dtype=np.float32, offset_bytes=4 * c * n) for c in chans])
    got_lk = np.stack([lk.download(n, dtype=np.uint8, offset_bytes=c * n) for c in chans])
    pll_mism = int(np.sum(got_out != ref_out) + np.sum(got_lk != ref_lk))
    assert pll_mism == 0, f"c4 PLL spot check: {pll_mism} outputs / lock flags differ"
    m = n
    # the serial kernel on the same data, for reference (one pass)
    pll_s = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                        f.BiquadD.LowPass(20000.0, 0.7)).design(rate, nch=nch)
    pll_s.set_stream(bank.stream())
    pll_s.set_time_parallel(-1)
    _, ms_serial = time_events(lambda: pll_s.process_dev(mf.ptr, n, n, out.ptr, lk.ptr, n),
                               bank.stream(), 1, 0, lambda: (bank.sync(), synchronize()))
    res = {"config": f"c4: 255-tap matched filter + PLL FM demod (src/main.rs:41-46), {nch} ch x 2^{args.c4_log2n}",
           "metric": "complex Msamples/s (input, all channels)", "value": round(units / (ms * 1e-3) / 1e6, 1),
           "roofline": roof(12, units, ms), "fir_ms": round(ms_fir, 3), "pll_ms": round(ms - ms_fir, 3),
           "pll_ns_per_sample_chain": round((ms - ms_fir) * 1e6 / n, 2),
           "pll_plan": {"segment": plan[0], "warm": plan[1], "segments_per_channel": tp_segments,
                        "segments_recomputed": tp_recomputed,
                        "phase_ms": {"pass1": round(ph[0], 3), "rerun": round(ph[1], 3), "walk": round(ph[2], 3)}},
           "pll_serial_ms": round(ms_serial, 3),
           "pll_serial_ns_per_sample_chain": round(ms_serial * 1e6 / n, 2),
           "note": "the PLL recurrence is serial per channel; time-parallel segments (speculative warm-up, exact verification, DESIGN.md 3.6) spread a channel over many SIMDs -- pll_ns_per_sample_chain is the wall time per sample of the whole batch",
           "wall_ms_per_step": round(wall * 1e3, 3), "fir_spot_check_max_over_rms": fir_check,
           "pll_spot_check": f"channels {chans} x {m} samples (the whole stream, time-parallel plan {plan}): outputs + lock flags array_equal to the oracle"}
    if not args.no_cpu_baseline:
        cores = min(os.cpu_count() or 1, 16)
        cn, cl = cores, 1 << 14
        xs = cplx_pattern(cn * cl, 8).reshape(cn, cl)
        p = pyoracle.pll_params(0.0, 0.035, rate, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
        t0, done = time.perf_counter(), 0
        while time.perf_counter() - t0 < args.cpu_seconds:
            m = pyoracle.fir_batch(taps, xs, 1, nthreads=cores)
            pyoracle.pll_batch(p, m, nthreads=cores)
            done += cn * cl
        el = time.perf_counter() - t0
        from bench import host_info
        res["cpu_baseline"] = {"value": round(done / el / 1e6, 2), "unit": "complex Msamples/s",
                               "cores": cores, "kind": "port", "host": host_info(),
                               "sample": f"{done} samples ({cn} ch x 2^14 blocks) oracle FIR+PLL, {el:.1f} s"}
    return res


# ------------------------------------------------------------------------------ c5
def bench_c5(args):
    """configs[4] through bench.channel_sharded_leg (the same leg bench.py adds to the
    driver's line): resident bank rate, RCCL scatterv / gatherv each timed on its own, end to
    end, and a float64 spot check of one channel per rank after the gather on the root."""
    import scipy.signal as ss
    import bench
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import sdrgpu
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, sdrgpu.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
        bench.init_gloo_quiet(dist)
    res = bench.channel_sharded_leg(args.steps, args.warmup, world, rank, local, dist,
                                    nch_total=args.c5_nch, log2n=args.c5_log2n, check=not args.no_check)
    res["config"] = res.pop("workload")
    res["metric"] = "complex Msamples/s (input, all ranks)"
    res["value"] = res["resident"]["value"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle
        taps = ss.firwin(255, 0.2).astype(np.float32)
        cores = min(os.cpu_count() or 1, 16)
        cn, cl = 4 * cores, 1 << 14
        xs = cplx_pattern(cn * cl, 9).reshape(cn, cl)
        t0, done = time.perf_counter(), 0
        while time.perf_counter() - t0 < args.cpu_seconds:
            pyoracle.fir_batch(taps, xs, 1, nthreads=cores)
            done += cn * cl
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(done / el / 1e6, 2), "unit": "complex Msamples/s",
                               "cores": cores, "kind": "port", "host": bench.host_info(),
                               "sample": f"{done} samples ({cn} ch x 2^14 blocks) through the "
                                         f"oracle Fir (255 taps, one Fir per channel), {el:.1f} s"}
    if dist is not None:
        dist.destroy_process_group()
    return res if rank == 0 else None


# ------------------------------------------------------------------------------ src
def bench_src(args):
    """src/main.rs:50's resample_with(SincFastest, 144 kHz) from 1.8 Msps (ratio 0.08) over a
    batch of 1024 complex streams (2048 interleaved channels), state carried call to call;
    the linear converter on the same shape; and one mono SincFastest stream (main.rs as
    written: a single FM audio channel), 4096-frame calls as adapters::Resample makes them."""
    import time as _t

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from sdrgpu import resample
    from sdrgpu.device import DeviceBuffer, synchronize
    ratio = float(np.float32(144000.0)) / float(np.float32(1.8e6))
    lines = []
    for conv, ch, nf in ((resample.ConverterType.Linear, 2048, 1 << 16),
                         (resample.ConverterType.SincFastest, 2048, 1 << 16),
                         (resample.ConverterType.SincFastest, 1, 4096)):
        g = resample.SampleRate(conv, ch)
        nfl = nf * ch
        x = DeviceBuffer.empty((nfl + 1) // 2)
        fill(x, (nfl + 1) // 2, 13)
        out_cap = int(nf * ratio) + 16
        y = DeviceBuffer.empty((out_cap * ch + 1) // 2)
        gen = [0]

        def step():  # state carries from call to call, as in a stream
            gen[0] = g.process_dev(ratio, x.ptr, nf, y.ptr, out_cap)[1]

        wall, ms = time_events(step, g.stream(), args.steps, args.warmup,
                               lambda: (g.sync(), synchronize()))
        nout = gen[0]
        name = "linear" if conv == resample.ConverterType.Linear else "SincFastest"
        line = {"config": f"src: {name} resampler 1.8 Msps -> 144 kHz (ratio 0.08), "
                          + (f"{ch // 2} complex streams = {ch} interleaved channels" if ch > 1
                             else "one mono stream (src/main.rs:50)") + f" x {nf} frames per call",
                "metric": "input Msamples/s (all channels)",
                "value": round(nfl / (ms * 1e-3) / 1e6, 1),
                "wall_value": round(nfl / wall / 1e6, 1),
                "output_frames": nout, "gpu_ms_per_call": round(ms, 4),
                "wall_ms_per_step": round(wall * 1e3, 3)}
        if conv == resample.ConverterType.Linear:
            line["roofline_kernel_estimate"] = roof(12, nout * ch, ms)
        else:
            c, inc = resample.sinc_table(conv)
            taps = 2 * (c.size - 2) / (inc * ratio)  # per output sample, both halves
            # per tap per output sample: one f64 multiply + one f64 add (the coefficient
            # interpolation is per frame, shared by the channels in the wide kernel)
            fl = 2 * taps * nout * ch / (ms * 1e-3) / 1e12
            line["taps_per_output"] = round(taps, 1)
            line["parity"] = ("unpinned vs libsamplerate: this library's own sinc tables "
                              "(DESIGN.md 3.7); bit-exact to the oracle restatement only")
            line["roofline"] = {"bound": "fp64 issue", "achieved": round(fl, 3),
                                "peak": 78.6, "unit": "TFLOP/s (f64 vector, AMD spec)",
                                "frac": round(fl / 78.6, 4)}
            if not args.no_cpu_baseline and ch == 1:
                xs = np.random.default_rng(1).standard_normal((nf, 1)).astype(np.float32)
                o = pyoracle.SampleRate(int(conv), 1)
                t0, done = _t.perf_counter(), 0
                while _t.perf_counter() - t0 < 3.0:
                    used, _ = o.process(ratio, xs, out_cap)
                    done += used
                dt = _t.perf_counter() - t0
                line["cpu_baseline"] = {"value": round(done / dt / 1e6, 3),
                                        "unit": "input Msamples/s", "cores": 1, "kind": "port",
                                        "sample": f"{done} mono samples through the oracle sinc, {dt:.1f} s"}
        lines.append(line)
    return lines


# ------------------------------------------------------------------------------ fm
def fm_stereo_u8(n, seed=0, rate=1.8e6):
    """A synthetic FM stereo broadcast as rtl_tcp u8 I/Q (the generator of
    tests/test_fm_chain_gpu.py): (L + R) + 0.1 pilot + (L - R) at 38 kHz DSB, 75 kHz deviation."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / rate
    left = 0.4 * np.sin(2 * np.pi * 440.0 * t)
    right = 0.4 * np.sin(2 * np.pi * 1250.0 * t + 0.3)
    comp = (0.45 * (left + right) + 0.1 * np.cos(2 * np.pi * 19000.0 * t)
            + 0.45 * (left - right) * np.cos(2 * np.pi * 38000.0 * t))
    iq = np.exp(1j * 2 * np.pi * 75000.0 * np.cumsum(comp) / rate) * 0.8
    iq = iq + 0.02 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    raw = np.empty(2 * n, np.uint8)
    raw[0::2] = np.clip(np.round(iq.real * 127.5 + 127.5), 0, 255).astype(np.uint8)
    raw[1::2] = np.clip(np.round(iq.imag * 127.5 + 127.5), 0, 255).astype(np.uint8)
    return raw


def bench_fm(args):
    """src/main.rs:33-81 end to end (sdrgpu.fm.receiver: PLL discriminator on the rtl_tcp bytes,
    SincFastest to 144 kHz, pilot-PLL stereo difference, SincBestQuality to 48 kHz, de-emphasis)
    over `--fm-seconds` of synthetic air in the reference's 0.1 s blocks (block(0.1), main.rs:47):
    seconds of air per second of wall time, host bytes in and audio out included (the chain's
    blocks come from and go to host memory, as main.rs's socket and WAV writer do).  The CPU
    baseline is the oracle's restatement of the same chain (tests/test_fm_chain_gpu.py's
    composition) on 1 s of air."""
    from sdrgpu import _lib, fm
    from sdrgpu.signal import from_array
    rate = fm.RATE
    n = int(rate * args.fm_seconds)
    raw = fm_stereo_u8(n)
    blk = int(rate * 0.1)
    warm = from_array(rate, raw[:2 * blk * 5], block=blk, sample_kind=_lib.CU8)
    list(fm.receiver(warm).blocks())
    rtl = from_array(rate, raw, block=blk, sample_kind=_lib.CU8)
    t0 = time.perf_counter()
    out = np.concatenate(list(fm.receiver(rtl).blocks()), axis=0)
    el = time.perf_counter() - t0
    res = {"config": "fm: src/main.rs FM stereo receiver chain, 1 station, u8 I/Q at 1.8 Msps in 0.1 s blocks",
           "metric": "seconds of air per second (real-time factor)",
           "value": round(args.fm_seconds / el, 1), "air_seconds": args.fm_seconds,
           "wall_s": round(el, 3), "audio_frames": int(out.shape[0]),
           "input_Msps": round(n / el / 1e6, 1)}
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import pyoracle
        from bench import host_info
        from test_fm_chain_gpu import oracle_chain
        cs = min(1.0, args.fm_seconds)
        t0 = time.perf_counter()
        oracle_chain(pyoracle, raw[:2 * int(rate * cs)], fm)
        ce = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(cs / ce, 2), "unit": "seconds of air per second",
                               "cores": 1, "kind": "port", "host": host_info(),
                               "sample": f"{cs:.1f} s of air through the oracle's chain, {ce:.1f} s"}
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.config != "c5":
            sys.exit("--gpus > 1 applies to --config c5 only")
        from bench import launch_ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], script=os.path.abspath(__file__)))
    todo = ["c1", "c3", "c4", "c5", "c2u8", "c2host", "c2pinned", "src", "ex", "fm"] if args.config == "all" else [args.config]
    for c in todo:
        r = {"c1": bench_c1, "c3": bench_c3, "c4": bench_c4, "c5": bench_c5, "c2u8": bench_c2u8,
             "c2host": bench_c2host, "c2pinned": bench_c2pinned, "src": bench_src, "ex": bench_ex,
             "fm": bench_fm}[c](args)
        for line in (r if isinstance(r, list) else [r]):
            if line is not None:
                print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
