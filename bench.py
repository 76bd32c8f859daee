#!/usr/bin/env python3
"""bench.py -- headline benchmark: complex Msamples/s through the 255-tap FIR on MI355X.

Workload (BASELINE.json configs[1]): 255-tap real-tap FIR, decimate by 4, over complex
f32 IQ (nominal 2.4 Msps stream -> 600 ksps), single channel per GPU, 2^28 input samples
per step, inputs resident in HBM.  One step = one sdrgpu_fir_process_dev() call over the
whole batch (the FIR state carries across steps, as a stream would).

Multi-GPU (one process per GPU): each rank filters its own time shard of the stream (weak
scaling; no data-path collective -- SURVEY.md 8e).  Under torch.distributed.run the ranks
come from the environment (WORLD_SIZE must equal --gpus); a plain `python bench.py --gpus
N` spawns the N rank processes itself (before anything touches the GPU) and relays rank
0's line.  Timing: barrier + synchronize on both sides of exactly K steps, MAX over ranks;
value = all ranks' samples / that time.

Also reported (rank 0, N=1 only unless --cpu-baseline force):
  roofline      algorithmic bytes per launch (10 B / input sample) / the
                kernel's average HIP-event-timed duration, vs 8 TB/s HBM3E;
  cpu_baseline  the oracle (C restatement of Fir::apply + Decimate, 1 core) on a bounded
                sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "unnamed-rust-sdr_amd"))

METRIC = "complex Msamples/sec through 255-tap FIR, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3
BYTES_PER_SAMPLE = 8 + 8 / 4   # c64 in + c64 out at decim 4
FLOPS_PER_SAMPLE = 255 * 4 / 4 # direct form, kept outputs only


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed steps (~0.1 s at configs[1]): the per-launch kernel time settles over the first
    # ~100 launches (0.513 ms mean over 20 steps, 0.500 over 100, 0.495 over 300 on one box,
    # profiles/r03_bench_steps.txt), and the fixed start/stop cost of the timed region is
    # amortised; 20 warmup steps
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--log2n", type=int, default=28, help="input samples per GPU per step")
    ap.add_argument("--algo", default="auto", choices=["auto", "direct", "os", "mx"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_fir_c2.json"))
    ap.add_argument("--leg-timeout", type=float, default=240.0,
                    help="seconds before a hung channel-sharded (RCCL) leg is abandoned")
    ap.add_argument("--no-channel-sharded", action="store_true",
                    help="skip the configs[4] channel-sharded FIR bank leg")
    return ap.parse_args()


def synth_iq_pattern(n, seed):
    """x = sum of 3 tones (random f in +-0.4 fs, amp 0.3) + 0.1 N(0,1), complex."""
    r = np.random.default_rng(seed)
    t = np.arange(n, dtype=np.float64)
    x = (r.standard_normal(n) + 1j * r.standard_normal(n)) * 0.1
    for f in r.uniform(-0.4, 0.4, 3):
        x += 0.3 * np.exp(2j * np.pi * np.remainder(f * t, 1.0))
    return x.astype(np.complex64)


def host_info():
    """Host CPU the baseline ran on (nproc and the /proc/cpuinfo model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"nproc": os.cpu_count(), "usable_cpus": usable, "cpu_model": model}


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None, timeout=1800.0):
    """Run `script argv` as n rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    set, rendezvous on 127.0.0.1), relay rank 0's output, return the first failing rank's
    exit status.  The parent never touches the GPU: every rank is a fresh process.  The
    children are polled together: when one exits non-zero the others are killed (a dead rank
    would otherwise leave the rest blocked in the rendezvous), and after `timeout` seconds
    all are killed and 124 is returned."""
    import threading
    script = script or os.path.abspath(__file__)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        failed = [c for c in codes if c not in (None, 0)]
        if failed:
            rc = failed[0]
            break
        if all(c == 0 for c in codes):
            break
        if deadline is not None and time.monotonic() > deadline:
            rc = 124
            break
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            p.kill()
    for p in procs:
        p.wait()
    reader.join(timeout=10)
    sys.stdout.write(b"".join(c for c in chunks if c).decode())
    sys.stdout.flush()
    return rc


def cpu_baseline(taps, seconds):
    """Oracle (restated reference path: all outputs computed, 3 of 4 dropped) on 1 core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    rng = np.random.default_rng(1)
    chunk = 1 << 18
    x = ((rng.standard_normal(chunk) + 1j * rng.standard_normal(chunk)) * 0.3).astype(np.complex64)
    f = pyoracle.Fir(taps, 4, sample_kind=1)
    done = 0
    t0 = time.perf_counter()
    while True:
        f.process(x)
        done += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el / 1e6, "unit": "complex Msamples/s", "cores": 1,
            "kind": "port", "host": host_info(),
            "sample": f"{done} c64 samples ({done // chunk} blocks of 2^18) through the oracle "
                      f"Fir(255 taps)+Decimate(4), {el:.1f} s on 1 host core"}


KERNEL_SOURCES = ("unnamed-rust-sdr_amd/csrc/fir_mxh.hip", "unnamed-rust-sdr_amd/csrc/fir_kernels.hpp")


def code_tokens(text):
    """C/C++ source with comments removed and whitespace runs collapsed: what the compiler
    sees, so a comment or layout edit does not change the hash below."""
    import re
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return " ".join(text.split())


def kernel_source_sha16(root=ROOT):
    """sha256[:16] over the headline kernel's source files (comments and layout stripped,
    code_tokens): ties a committed PMC traffic figure to the kernel code it was measured on
    (tools/pmc_to_json.py records it)."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(root, rel)) as f:
            h.update(code_tokens(f.read()).encode())
    return h.hexdigest()[:16]


def pmc_traffic(path, log2n, algo):
    """(traffic bytes per launch or None, traffic_source) from the committed PMC file; the
    figure is used only when it was measured on this exact kernel source and workload."""
    src = {"file": os.path.relpath(path, ROOT), "kernel_source_sha16": kernel_source_sha16()}
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        src["status"] = "missing"
        return None, src
    src.update({"measured_sha16": pm.get("kernel_source_sha16"), "method": pm.get("method"),
                "commit": pm.get("commit")})
    if pm.get("log2n") != log2n or pm.get("algo", "auto") != algo:
        src["status"] = "other workload"
        return None, src
    if pm.get("kernel_source_sha16") != src["kernel_source_sha16"]:
        src["status"] = "stale: measured on another kernel source"
        return None, src
    src["status"] = "matches this kernel source"
    return pm.get("hbm_bytes_per_launch"), src


def channel_block_bytes(nch_total, world, n):
    """Per-rank byte counts of the channel blocks scatterv / gatherv move (c64 channels of n
    samples, split by sdrgpu.shard.channel_range; zero for ranks with no channel)."""
    from sdrgpu.shard import channel_range
    return [(b - a) * n * 8 for a, b in (channel_range(nch_total, world, r) for r in range(world))]


def channel_offset_bytes(c, n):
    """Byte offset of channel c in the root's packed all-channel buffer (the layout scatterv /
    gatherv use: rank blocks in rank order, channels contiguous inside a block)."""
    return 8 * c * n


def channel_sharded_leg(steps, warmup, world, rank, local, dist, nch_total=8192, log2n=16, check=True):
    """configs[4] / north_star's multi-GPU claim, measured in the line the driver runs: an
    8192-channel x 2^16 c64 255-tap FIR bank (D = 1) with its channels sharded over the
    ranks (sdrgpu.shard.channel_range, one process per GPU).  Reported separately:
      resident   every rank filters its own resident channel block (weak scaling of the
                 bank: the per-step time is the max over ranks, the rate counts all channels);
      rccl       the fan-out of the channel blocks from rank 0 (scatterv) and the gather of
                 the outputs back (gatherv) over xGMI, each timed on its own (HIP events on the
                 bank's stream, max over ranks);
      end_to_end all channels / (scatter + one resident step + gather);
      spot_check on rank 0 after the gather, one channel of EVERY rank's block against a
                 float64 NumPy FIR of its input (src/filter/fir.rs:23-32 per channel).
    Ranks sharing a GPU (a rehearsal on a smaller box) skip RCCL, which needs one device per
    rank."""
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu.device import DeviceBuffer, Event, synchronize
    from sdrgpu.shard import Comm, channel_range, unique_id
    n = 1 << log2n
    K = 255
    taps = ss.firwin(K, 0.2).astype(np.float32)
    lo, hi = channel_range(nch_total, world, rank)
    nch = hi - lo
    shared = world > sdrgpu.device_count()
    bank = sdrgpu.filter.FirBank(taps, nch, sample_kind=sdrgpu.C64, device=local)
    s = bank.stream()
    x = DeviceBuffer.empty(nch * n, np.complex64, device=local)
    y = DeviceBuffer.empty(nch * n, np.complex64, device=local)
    sizes = channel_block_bytes(nch_total, world, n)
    pat = synth_iq_pattern(1 << 22, seed=4000)
    use_rccl = world > 1 and not shared
    full_in = full_out = comm = None
    if rank == 0 and (use_rccl or world == 1):
        tgt = DeviceBuffer.empty(nch_total * n, np.complex64, device=local) if use_rccl else x
        for off in range(0, nch_total * n, pat.size):
            tgt.upload(pat[:min(pat.size, nch_total * n - off)], offset_bytes=8 * off)
        full_in = tgt
        full_out = DeviceBuffer.empty(nch_total * n, np.complex64, device=local) if use_rccl else y
    elif not use_rccl:  # shared-GPU rehearsal: each rank fills its own block
        for off in range(0, nch * n, pat.size):
            x.upload(pat[:min(pat.size, nch * n - off)], offset_bytes=8 * off)
    res = {"workload": f"configs[4]: {nch_total}-channel x 2^{log2n} c64 255-tap FIR bank (D=1), "
                       "channels sharded over the ranks, one GPU per rank",
           "channels_per_rank": [b - a for a, b in (channel_range(nch_total, world, r)
                                                    for r in range(world))]}
    if use_rccl:
        ids = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        comm = Comm(local, world, rank, ids[0])

        def coll(fn):  # one collective on the bank's stream, timed by events, max over ranks
            import torch
            e0, e1 = Event(local), Event(local)
            comm.barrier(s)
            e0.record(s)
            fn()
            e1.record(s)
            bank.sync()
            t = torch.tensor([e0.elapsed_ms(e1)], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
        scat = lambda: comm.scatterv(full_in.ptr if full_in else None, x.ptr, sizes, 0, s)
        gath = lambda: comm.gatherv(y.ptr, full_out.ptr if full_out else None, sizes, 0, s)
        coll(scat)  # warm-up (RCCL connection setup)
        scatter_ms = float(np.mean([coll(scat) for _ in range(3)]))
    synchronize(local)

    def step():
        bank.process_dev(x.ptr, n, n, y.ptr, n)

    def sync():
        bank.sync()
        synchronize(local)

    el = timed_region(step, steps, warmup, sync, dist if world > 1 else None)
    ms = el / steps * 1e3
    res["resident"] = {"value": round(nch_total * n / (ms * 1e-3) / 1e6, 1) if not shared else None,
                       "unit": "complex Msamples/s (all ranks)", "ms_per_step": round(ms, 4),
                       "roofline_frac_per_gpu": round(16 * nch * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if shared:
        res["rccl"] = "skipped: ranks share a GPU (RCCL needs one device per rank)"
        res["note"] = "shared-GPU rehearsal: not a throughput result"
    if use_rccl:
        coll(gath)
        gather_ms = float(np.mean([coll(gath) for _ in range(3)]))
        res["rccl"] = {"scatterv_ms": round(scatter_ms, 3), "gatherv_ms": round(gather_ms, 3),
                       "scatterv_GBps_root": round(sum(sizes[1:]) / (scatter_ms * 1e-3) / 1e9, 1),
                       "gatherv_GBps_root": round(sum(sizes[1:]) / (gather_ms * 1e-3) / 1e9, 1)}
        res["end_to_end"] = {"value": round(nch_total * n / ((scatter_ms + ms + gather_ms) * 1e-3) / 1e6, 1),
                             "unit": "complex Msamples/s", "ms": round(scatter_ms + ms + gather_ms, 3)}
        comm.close()
    if rank == 0 and full_out is not None:
        # steady state: every step filtered the same resident block, so a channel's history
        # entering the last step is the block's own last K-1 samples
        checks = {}
        m = 4096
        for r in range(world):
            a, b = channel_range(nch_total, world, r)
            c = (a + b) // 2
            xin = full_in.download(n, offset_bytes=channel_offset_bytes(c, n)).astype(np.complex128)
            ref = np.convolve(np.concatenate([xin[n - (K - 1):], xin[:m]]),
                              taps.astype(np.float64))[K - 1:K - 1 + m]
            got = full_out.download(m, offset_bytes=channel_offset_bytes(c, n))
            err = float(np.abs(got - ref).max() / np.sqrt(np.mean(np.abs(ref) ** 2)))
            checks[str(c)] = err
            assert err <= 1e-5 or not check, (c, err)
        res["spot_check_max_over_rms"] = checks
    return res


def init_gloo_quiet(dist):
    """dist.init_process_group("gloo") with file descriptor 1 pointed at stderr meanwhile: gloo
    prints "[Gloo] Rank r is connected to ..." on stdout, and the driver reads rank 0's stdout
    for the ONE JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        dist.init_process_group("gloo")
    finally:
        os.dup2(saved, 1)
        os.close(saved)


LEG_HUNG_EXIT = 3  # exit status of a rank whose channel-sharded leg hung (run_guarded)


def run_guarded(fn, seconds, rank, on_timeout):
    """Run the channel-sharded leg so that it cannot take the headline line down with it.  Its
    multi-rank RCCL part only runs on a node with one GPU per rank, so a failure there must not
    cost the configs[1] result: an exception becomes {"error": ...} in the line, and a hang (a
    peer that died inside a collective) fires a per-rank watchdog after `seconds` that calls
    on_timeout() (rank 0 prints the line with channel_sharded.error) and ends the process with
    status LEG_HUNG_EXIT, so every rank of the launch exits instead of waiting on the others and
    the hang shows up as a FAILED run (the launcher and the driver see the non-zero status) --
    the main thread may still be stuck inside a collective or a GPU call at that point."""
    import threading

    def fire():
        sys.stderr.write(f"bench.py rank {rank}: channel-sharded leg still running after {seconds:.0f} s; "
                         "abandoning it\n")
        try:
            on_timeout()
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(LEG_HUNG_EXIT)

    timer = threading.Timer(seconds, fire)
    timer.daemon = True
    timer.start()
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 -- reported in the line, never fatal to it
        sys.stderr.write(f"bench.py rank {rank}: channel-sharded leg failed: {e!r}\n")
        return {"error": repr(e)[:300]}
    finally:
        timer.cancel()


def headline_record(value, world, steps, warmup, elapsed, n, D, kern_ms, traffic, traffic_src,
                    algo):
    """The driver's JSON line (bench contract) for configs[1]; pure host logic (tested on
    CPU by tests/test_bench_cpu.py)."""
    achieved = BYTES_PER_SAMPLE * n / (kern_ms * 1e-3) / 1e9
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "complex Msamples/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: 3 tones + 0.1 N(0,1) complex64, 2^22-sample pattern per rank tiled to the shard",
        "config": {
            "workload": "configs[1]: 255-tap FIR (real f32 taps, firwin 0.2) decimate-by-4 "
                        "on complex IQ, single channel per GPU",
            "samples_per_gpu_per_step": n,
            "ntaps": 255, "decim": D, "sample": "c64", "taps": "f32",
            "algorithm": algo,
            "arith": "f32 samples and taps; on the default (MFMA) path each product is an "
                     "fp16x2 split of the samples (per-tile power-of-two scale) times an "
                     "fp16x2 split of the taps on v_mfma_f32_16x16x32_f16, f32 accumulate "
                     "(DESIGN.md 3.1; within north_star's 1e-5)",
            "parallelism": f"{world} time shards, no data-path collective",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel_ms": round(kern_ms, 4),
            "algorithmic_bytes_per_launch": int(BYTES_PER_SAMPLE * n),
            "fp32_tflops_direct_equiv": round(FLOPS_PER_SAMPLE * n / (kern_ms * 1e-3) / 1e12, 2),
        },
    }
    return res


def timed_region(step, steps, warmup, sync, dist=None, on_step=None):
    """Run `warmup` untimed steps, then exactly `steps` timed steps bracketed by a barrier
    and a device synchronize on both sides; return the MAX elapsed seconds over ranks.
    `on_step(i, phase)` is called with phase 'begin'/'end' around each timed step (event
    recording).  Pure host logic: tests/test_dist_cpu.py drives it with gloo ranks."""
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        if on_step:
            on_step(i, "begin")
        step()
        if on_step:
            on_step(i, "end")
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        # rank coordination only (barrier, max-time): the path has no data exchange, so
        # no RCCL collective is used; gloo keeps torch's own HIP runtime off the GPU.
        import torch.distributed as dist
        init_gloo_quiet(dist)

    import scipy.signal as ss
    import sdrgpu
    from sdrgpu import _lib
    from sdrgpu.device import DeviceBuffer, Event, synchronize

    # one GPU per rank; ranks beyond the visible GPUs share them round-robin (a rehearsal
    # of the N-rank path on a smaller box -- on a full node local < device_count)
    local = local % max(1, sdrgpu.device_count())
    taps = ss.firwin(255, 0.2).astype(np.float32)
    n = 1 << args.log2n
    D = 4
    algo = {"auto": _lib.FIR_AUTO, "direct": _lib.FIR_DIRECT, "os": _lib.FIR_OVERLAP_SAVE,
            "mx": _lib.FIR_MATRIX}[args.algo]
    fir = sdrgpu.filter.Fir(taps, decim=D, sample_kind=_lib.C64, device=local,
                            algorithm=algo).design(2.4e6)
    stream = fir.stream()

    # This rank's time shard of one long stream: shard r covers stream samples
    # [r*n, (r+1)*n).  Synthetic data: a 2^22-sample pattern (distinct per rank) tiled.
    pat_n = min(n, 1 << 22)
    pat = synth_iq_pattern(pat_n, seed=1000 + rank)
    x = DeviceBuffer.empty(n, np.complex64, device=local)
    for off in range(0, n, pat_n):
        x.upload(pat[:min(pat_n, n - off)], offset_bytes=8 * off)
    n_out = n // D
    y = DeviceBuffer.empty(n_out, np.complex64, device=local)
    if rank > 0:
        # halo: the 256 stream samples preceding this shard (tail of rank-1's shard) prime
        # the FIR history, so the sharded outputs equal the unsharded stream's exactly
        prev = synth_iq_pattern(pat_n, seed=1000 + rank - 1)
        halo = prev[(n - 256) % pat_n:][:256] if pat_n >= 256 else prev
        hb = DeviceBuffer.from_numpy(np.ascontiguousarray(halo), device=local)
        hy = DeviceBuffer.empty(64, np.complex64, device=local)
        fir.process_dev(hb.ptr, 256, hy.ptr, 64)
    synchronize(local)

    def step():
        got = fir.process_dev(x.ptr, n, y.ptr, n_out)
        assert got == n_out, (got, n_out)

    starts = [Event(local) for _ in range(args.steps)]
    ends = [Event(local) for _ in range(args.steps)]

    def on_step(i, phase):
        (starts if phase == "begin" else ends)[i].record(stream)

    def sync():
        fir.sync()
        synchronize(local)

    elapsed = timed_region(step, args.steps, args.warmup, sync, dist, on_step)
    kern_ms = float(np.mean([s.elapsed_ms(e) for s, e in zip(starts, ends)]))
    total_samples = n * args.steps * world
    value = total_samples / elapsed / 1e6
    if rank == 0:
        traffic, traffic_src = pmc_traffic(args.pmc_json, args.log2n, args.algo)
        res = headline_record(value, world, args.steps, args.warmup, elapsed, n, D, kern_ms,
                              traffic, traffic_src, args.algo)
    if not args.no_channel_sharded:
        def abandon():
            if rank == 0:
                res["channel_sharded"] = {"error": f"abandoned after {args.leg_timeout:.0f} s (RCCL leg hung)"}
                print(json.dumps(res), flush=True)
        cs = run_guarded(lambda: channel_sharded_leg(args.steps, args.warmup, world, rank, local, dist),
                         args.leg_timeout, rank, abandon)
    if rank == 0:
        if not args.no_channel_sharded:
            res["channel_sharded"] = cs
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(taps, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
