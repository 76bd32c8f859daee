"""Dump the FIR outputs of tests/test_fir_gpu.py::test_fir_mx_silent_stretches' inputs (and the
oracle's) for offline study of the per-window errors.  Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "unnamed-rust-sdr_amd")]
import pyoracle  # noqa: E402
import sdrgpu  # noqa: E402
import test_fir_gpu as T  # noqa: E402

out = {}


class Cap:
    def __init__(self, real):
        self.real = real

    def __getattr__(self, k):
        return getattr(self.real, k)


class FirWrap:
    def __init__(self, key):
        self.key = key

    def __call__(self, taps, decim, sample_kind):
        d = sdrgpu.filter.Fir(taps, decim=decim, sample_kind=sample_kind)

        class D:
            def design(_, rate):
                h = d.design(rate)

                class H:
                    def process(_, inp):
                        y = h.process(inp)
                        out[self.key + "_y"] = y
                        out[self.key + "_in"] = inp
                        out[self.key + "_taps"] = taps
                        return y

                    def last_kernel(_):
                        return h.last_kernel()
                return H()
        return D()


class Sdr:
    pass


for sk, D in [(1, 4), (1, 1), (2, 4)]:
    key = f"sk{sk}D{D}"
    s = Sdr()
    s.filter = type("F", (), {"Fir": staticmethod(FirWrap(key))})
    try:
        T.test_fir_mx_silent_stretches(s, pyoracle, sk, D)
        print(key, "passed")
    except AssertionError as e:
        print(key, "FAILED", str(e).splitlines()[0])
os.makedirs(os.path.join(ROOT, "gpurun_out", "r06_silent"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "r06_silent", "dump.npz"), **out)
