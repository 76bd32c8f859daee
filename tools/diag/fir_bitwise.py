"""Dump the MFMA FIR paths' outputs on seeded inputs, for a bitwise comparison of two builds
(diagnostic, not a test):
    python tools/experiments/run_with_lib.py A.so tools/diag/fir_bitwise.py OUT_A.npz
    python tools/diag/fir_bitwise.py OUT_B.npz          # the product library
    python tools/diag/fir_bitwise.py --compare OUT_A.npz OUT_B.npz
Inputs: complex noise whose block amplitude jumps over 2^-30 .. 2^30 (every per-tile scale,
the sticky-scale cases on both sides of a power of two, the fp16-subnormal tail, exact-zero
stretches), plus a run of samples just below / above 2^k boundaries.  Cases: c64 D = 4 (255 taps, the headline
kernel), D = 2, the D = 1 bank, several streamed blocks each."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def signal(n, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    blk = 1024 + 37
    e = rng.integers(-30, 31, size=n // blk + 1)
    amp = np.repeat(np.exp2(e.astype(np.float64)), blk)[:n]
    # slow drifts across a power of two (window max just below / above 2^k)
    drift = np.exp2(0.6 * np.sin(np.arange(n) * 2 * np.pi / 50000.0))
    x = (x * (amp * drift)).astype(np.complex64)
    edge = rng.integers(0, n - 4096)
    x[edge:edge + 4096] = np.float32(65504.0) * np.sign(x[edge:edge + 4096].real) + 1j * np.float32(1.5)
    # exact silence: all-zero tiles and the sticky-scale choice of the tile after them
    for z in rng.integers(0, n - 5000, size=3):
        x[z:z + int(rng.integers(300, 5000))] = 0
    return x


def run(out):
    sys.path.insert(0, os.path.join(ROOT, "unnamed-rust-sdr_amd"))
    import scipy.signal as ss
    import sdrgpu
    from sdrgpu import _lib
    taps = ss.firwin(255, 0.2).astype(np.float32)
    res = {}
    for D in (4, 2):
        f = sdrgpu.filter.Fir(taps, decim=D, sample_kind=_lib.C64).design(2.4e6)
        x = signal(1 << 21, 10 + D)
        ys = [f.process(x[a:b]) for a, b in ((0, 700001), (700001, 700001 + 2048), (702049, 1 << 21))]
        res[f"d{D}"] = np.concatenate(ys)
        res[f"d{D}_kernel"] = np.array([f.last_kernel()])
    nch, n = 64, 1 << 15
    bank = sdrgpu.filter.FirBank(taps, nch, sample_kind=_lib.C64)
    xb = signal(nch * n, 99).reshape(nch, n)
    res["bank"] = np.concatenate([bank.process(xb[:, :12345]), bank.process(xb[:, 12345:])], axis=1)
    np.savez(out, **res)
    print(out, {k: v.shape for k, v in res.items()})


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        va, vb = A[k], B[k]
        same = va.shape == vb.shape and np.array_equal(va.view(np.uint8), vb.view(np.uint8))
        nd = 0 if same else int(np.count_nonzero(va.view(np.uint32) != vb.view(np.uint32)))
        print(f"{k:12s} {va.shape} {'bit-identical' if same else f'{nd} words differ'}")
        bad += not same
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
    run(sys.argv[1])
