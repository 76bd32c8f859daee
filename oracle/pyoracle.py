"""ctypes access to liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
See oracle.h for what is restated (reference file:line) and the parity status.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_size_t, c_uint32, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

F32, C64 = 0, 1
BQ_IDENTITY, BQ_LOWPASS, BQ_HIGHPASS, BQ_BANDPASS, BQ_NOTCH, BQ_LR = range(6)


class BiquadDesign(ctypes.Structure):
    _fields_ = [("kind", c_int), ("freq", c_float), ("q", c_float)]


class BiquadCoefs(ctypes.Structure):
    _fields_ = [("b0", c_float), ("b1", c_float), ("b2", c_float), ("na1", c_float),
                ("na2", c_float)]


class PllParams(ctypes.Structure):
    _fields_ = [("reference", c_float), ("gain", c_float), ("rate", c_float),
                ("loopf", BiquadDesign), ("outputf", BiquadDesign), ("lockf", BiquadDesign)]


_L = None


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_fir_create.restype = c_void_p
        L.oracle_fir_create.argtypes = [c_int, c_int, c_void_p, c_size_t, c_uint32]
        L.oracle_fir_destroy.argtypes = [c_void_p]
        L.oracle_fir_reset.argtypes = [c_void_p]
        L.oracle_fir_process.restype = c_size_t
        L.oracle_fir_process.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p]
        L.oracle_fir_batch.restype = c_size_t
        L.oracle_fir_batch.argtypes = [c_int, c_int, c_void_p, c_size_t, c_uint32, c_size_t,
                                       c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, c_int]
        L.oracle_biquad_design_coefs.argtypes = [BiquadDesign, c_float, POINTER(BiquadCoefs)]
        L.oracle_biquad_run.argtypes = [BiquadDesign, c_float, c_int, c_void_p, c_size_t,
                                        c_void_p]
        L.oracle_pll_batch.argtypes = [POINTER(PllParams), c_size_t, c_void_p, c_size_t,
                                       c_size_t, c_void_p, c_void_p, c_size_t, c_int]
        L.oracle_pll_stereo.argtypes = [POINTER(PllParams), c_void_p, c_size_t, c_void_p,
                                         c_void_p, c_void_p]
        L.oracle_fft_frame.argtypes = [c_void_p, c_size_t, c_void_p]
        L.oracle_stft.restype = c_size_t
        L.oracle_stft.argtypes = [c_void_p, c_size_t, c_size_t, c_size_t, c_void_p, c_size_t,
                                  c_int]
        L.oracle_freq.argtypes = [c_float, c_float, c_float, c_size_t, c_void_p]
        L.oracle_freq_sweep.restype = c_size_t
        L.oracle_freq_sweep.argtypes = [c_float, c_float, c_int, c_float, c_float, c_size_t,
                                        c_void_p, c_void_p]
        L.oracle_u8_to_c64.argtypes = [c_void_p, c_size_t, c_void_p]
        L.oracle_libm.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]
        L.oracle_src_new.restype = c_void_p
        L.oracle_src_new.argtypes = [c_int, c_int, POINTER(c_int)]
        L.oracle_src_delete.argtypes = [c_void_p]
        L.oracle_sinc_table.argtypes = [c_int, c_void_p, c_int, POINTER(c_int)]
        L.oracle_src_reset.argtypes = [c_void_p]
        L.oracle_src_set_ratio.argtypes = [c_void_p, ctypes.c_double]
        L.oracle_src_process.argtypes = [c_void_p, c_void_p, ctypes.c_long, c_void_p,
                                         ctypes.c_long, ctypes.c_double,
                                         POINTER(ctypes.c_long), POINTER(ctypes.c_long)]
        _L = L
    return _L


def _kind(a):
    return C64 if np.iscomplexobj(a) else F32


class Fir:
    """Streaming Fir + Decimate restatement (fir.rs:23-32, adapters/mod.rs:30-37)."""

    def __init__(self, taps, decim=1, sample_kind=None):
        taps = np.asarray(taps)
        self.tk = _kind(taps)
        self.taps = np.ascontiguousarray(taps, np.complex64 if self.tk else np.float32)
        self.sk = sample_kind if sample_kind is not None else self.tk
        self.decim = decim
        self.h = lib().oracle_fir_create(self.sk, self.tk, self.taps.ctypes.data,
                                         self.taps.size, decim)
        if not self.h:
            raise ValueError("oracle_fir_create rejected the configuration")

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_fir_destroy(self.h)
            self.h = None

    def reset(self):
        lib().oracle_fir_reset(self.h)

    def process(self, x):
        dt = np.complex64 if self.sk else np.float32
        x = np.ascontiguousarray(x, dt)
        out = np.empty(x.size // self.decim + 1, dt)
        n = lib().oracle_fir_process(self.h, x.ctypes.data, x.size, out.ctypes.data)
        return out[:n]


def fir_batch(taps, x, decim=1, nthreads=1):
    taps = np.asarray(taps)
    tk = _kind(taps)
    taps = np.ascontiguousarray(taps, np.complex64 if tk else np.float32)
    sk = _kind(x)
    dt = np.complex64 if sk else np.float32
    x = np.ascontiguousarray(x, dt)
    nch, n = x.shape
    out = np.empty((nch, n // decim + 1), dt)
    n_out = lib().oracle_fir_batch(sk, tk, taps.ctypes.data, taps.size, decim, nch,
                                   x.ctypes.data, n, n, out.ctypes.data, out.shape[1],
                                   nthreads)
    return out[:, :n_out]


def biquad_coefs(kind, freq, q, rate):
    c = BiquadCoefs()
    lib().oracle_biquad_design_coefs(BiquadDesign(kind, freq, q), rate, ctypes.byref(c))
    return (c.b0, c.b1, c.b2, c.na1, c.na2)


def biquad_run(kind, freq, q, rate, x):
    sk = _kind(x)
    dt = np.complex64 if sk else np.float32
    x = np.ascontiguousarray(x, dt)
    out = np.empty_like(x)
    lib().oracle_biquad_run(BiquadDesign(kind, freq, q), rate, sk, x.ctypes.data, x.size,
                            out.ctypes.data)
    return out


def pll_params(reference, gain, rate, loopf, outputf, lockf):
    return PllParams(reference, gain, rate, BiquadDesign(*loopf), BiquadDesign(*outputf),
                     BiquadDesign(*lockf))


def pll_batch(params, x, nthreads=1):
    x = np.ascontiguousarray(x, np.complex64)
    if x.ndim == 1:
        x = x[None, :]
    nch, n = x.shape
    out = np.empty((nch, n), np.float32)
    locked = np.empty((nch, n), np.uint8)
    lib().oracle_pll_batch(ctypes.byref(params), nch, x.ctypes.data, n, n, out.ctypes.data,
                           locked.ctypes.data, n, nthreads)
    return out, locked


def pll_stereo(params, v):
    v = np.ascontiguousarray(v, np.float32)
    mono, diff = np.empty_like(v), np.empty_like(v)
    locked = np.empty(v.size, np.uint8)
    lib().oracle_pll_stereo(ctypes.byref(params), v.ctypes.data, v.size, mono.ctypes.data,
                            diff.ctypes.data, locked.ctypes.data)
    return mono, diff, locked


def fft_frame(x):
    x = np.ascontiguousarray(x, np.complex64)
    out = np.empty_like(x)
    lib().oracle_fft_frame(x.ctypes.data, x.size, out.ctypes.data)
    return out


def stft(x, n, hop, max_frames=None, nthreads=1):
    x = np.ascontiguousarray(x, np.complex64)
    nf = x.size // hop
    if max_frames is not None:
        nf = min(nf, max_frames)
    out = np.empty((nf, n), np.complex64)
    got = lib().oracle_stft(x.ctypes.data, x.size, n, hop, out.ctypes.data, nf, nthreads)
    return out[:got]


def freq(rate, f, phase, n):
    out = np.empty(n, np.complex64)
    lib().oracle_freq(rate, f, phase, n, out.ctypes.data)
    return out


def freq_sweep(rate, df, warmup, start, end):
    """(freqs f32, values c64) of freq_sweep(rate, df, warmup, start..end) (sources.rs:181-194)."""
    n = lib().oracle_freq_sweep(rate, df, int(warmup), start, end, 0, None, None)
    f = np.empty(n, np.float32)
    v = np.empty(n, np.complex64)
    lib().oracle_freq_sweep(rate, df, int(warmup), start, end, n, f.ctypes.data, v.ctypes.data)
    return f, v


def u8_to_c64(iq_u8):
    iq_u8 = np.ascontiguousarray(iq_u8, np.uint8)
    out = np.empty(iq_u8.size // 2, np.complex64)
    lib().oracle_u8_to_c64(iq_u8.ctypes.data, out.size, out.ctypes.data)
    return out


def atan2f(y, x):
    """glibc atan2f elementwise (f32)."""
    y = np.ascontiguousarray(y, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(y)
    lib().oracle_libm(0, y.ctypes.data, x.ctypes.data, out.ctypes.data, None, y.size)
    return out


def sincosf(a):
    """glibc (sinf(a), cosf(a)) elementwise (f32)."""
    a = np.ascontiguousarray(a, np.float32)
    s, c = np.empty_like(a), np.empty_like(a)
    lib().oracle_libm(1, a.ctypes.data, None, s.ctypes.data, c.ctypes.data, a.size)
    return s, c


def sinc_table(converter):
    """(coefficients f32, increment) of sinc converter 0/1/2 (oracle_sinc_table)."""
    inc = c_int(0)
    n = lib().oracle_sinc_table(converter, None, 0, ctypes.byref(inc))
    out = np.empty(n, np.float32)
    lib().oracle_sinc_table(converter, out.ctypes.data, n, ctypes.byref(inc))
    return out, inc.value


class SampleRate:
    """libsamplerate sinc / ZOH / linear restatement behind SampleRate (src/resample.rs:32-110).

    `process(ratio, frames)` takes a (n, channels) float32 array and returns
    (input_frames_used, output (m, channels)), like SampleRate::process with an output
    capacity of `out_cap` frames."""

    def __init__(self, converter, channels):
        err = c_int(0)
        self.channels = channels
        self.h = lib().oracle_src_new(converter, channels, ctypes.byref(err))
        if not self.h:
            raise ValueError(f"oracle_src_new: libsamplerate error {err.value}")

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_src_delete(self.h)
            self.h = None

    def reset(self):
        lib().oracle_src_reset(self.h)

    def set_ratio(self, ratio):
        return lib().oracle_src_set_ratio(self.h, ratio)

    def process(self, ratio, frames, out_cap):
        x = np.ascontiguousarray(frames, np.float32).reshape(-1, self.channels)
        out = np.zeros((max(out_cap, 1), self.channels), np.float32)
        used, gen = ctypes.c_long(0), ctypes.c_long(0)
        rc = lib().oracle_src_process(self.h, x.ctypes.data if x.size else None, x.shape[0],
                                      out.ctypes.data, out_cap, ratio, ctypes.byref(used),
                                      ctypes.byref(gen))
        if rc:
            raise ValueError(f"oracle_src_process: libsamplerate error {rc}")
        return used.value, out[:gen.value].copy()
