"""Host-side mirror of the reference `fft` module (src/fft.rs) over the sdrgpu C ABI.

  fft::fft(signal)  -> Vec<(f32, Complex<f32>)>   src/fft.rs:3-28
  fft::rfft(signal) -> Vec<(f32, Complex<f32>)>   src/fft.rs:30-37

`fft(x, rate)` / `rfft(x, rate)` return (freqs, values) arrays instead of a Vec of tuples;
values are the collated, 1/sqrt(N)-normalised spectrum exactly as the reference orders it.
`Stft` is the streaming composition sig.window(N/rate).decimate(rate/hop).map(fft::fft)
(examples/live.rs:29-39).  Any N >= 1 plans, like rustfft (fft.rs:10-11): powers of two on
the Stockham / four-step kernels, other lengths on mixed-radix tiles or Bluestein.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from ._lib import check, lib


def freqs(n: int, rate: float) -> np.ndarray:
    out = np.empty(n, np.float32)
    check(lib().sdrgpu_fft_freqs(n, rate, out.ctypes.data), "sdrgpu_fft_freqs")
    return out


def _out_mode(output: str) -> int:
    if output not in ("complex", "db"):
        raise _lib.SdrGpuError(_lib.ERR_INVALID, "output must be 'complex' or 'db'")
    return _lib.FFT_OUT_DB if output == "db" else _lib.FFT_OUT_COMPLEX


class FftPlan:
    """A planned N-point forward FFT with fft.rs collation (plan once, unlike fft.rs:10-11).

    output='db' returns f32 20*log10(|value|) per bin instead of the complex value -- the
    spectrum plots' conversion (src/plot/complexseries.rs:90-92) fused into the store."""

    def __init__(self, n: int, device: int = 0, output: str = "complex"):
        self.n = int(n)
        self.device = device
        self.output = output
        self._h = ctypes.c_void_p()
        check(lib().sdrgpu_fft_plan(device, self.n, ctypes.byref(self._h)), "sdrgpu_fft_plan")
        check(lib().sdrgpu_fft_set_output(self._h, _out_mode(output)), "sdrgpu_fft_set_output")
        self._odt = np.float32 if output == "db" else np.complex64

    def close(self):
        if self._h:
            lib().sdrgpu_fft_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().sdrgpu_fft_get_stream(self._h, ctypes.byref(s)), "get_stream")
        return s.value or 0

    def exec(self, x) -> np.ndarray:
        """x: (count, n) or (n,) complex -> collated spectra of the same shape."""
        x = np.ascontiguousarray(x, np.complex64)
        squeeze = x.ndim == 1
        x2 = x.reshape(-1, self.n)
        out = np.empty(x2.shape, self._odt)
        check(lib().sdrgpu_fft_exec(self._h, x2.ctypes.data, out.ctypes.data, x2.shape[0]),
              "sdrgpu_fft_exec")
        return out[0] if squeeze else out

    def exec_real(self, x) -> np.ndarray:
        """rfft frames: (count, n) real -> (count, n - n/2) entries [n/2, n) of the collated
        output (fft.rs:35 drains the first n/2)."""
        x = np.ascontiguousarray(x, np.float32)
        squeeze = x.ndim == 1
        x2 = x.reshape(-1, self.n)
        out = np.empty((x2.shape[0], self.n - self.n // 2), self._odt)
        check(lib().sdrgpu_rfft_exec(self._h, x2.ctypes.data, out.ctypes.data, x2.shape[0]),
              "sdrgpu_rfft_exec")
        return out[0] if squeeze else out

    def exec_dev(self, d_in: int, d_out: int, count: int):
        check(lib().sdrgpu_fft_exec_dev(self._h, d_in, d_out, count), "sdrgpu_fft_exec_dev")

    def exec_real_dev(self, d_in: int, d_out: int, count: int):
        """rfft of `count` device-resident frames (n f32 each) -> n - n/2 outputs per frame."""
        check(lib().sdrgpu_rfft_exec_dev(self._h, d_in, d_out, count), "sdrgpu_rfft_exec_dev")

    def sync(self):
        check(lib().sdrgpu_fft_sync(self._h), "sdrgpu_fft_sync")


def fft(x, rate: float, device: int = 0):
    """fft::fft (fft.rs:3-28) of one finite complex signal: (freqs, values)."""
    x = np.ascontiguousarray(x, np.complex64)
    p = FftPlan(x.size, device)
    return freqs(x.size, rate), p.exec(x)


def rfft(x, rate: float, device: int = 0):
    """fft::rfft (fft.rs:30-37): real input, keeps the upper half of the collated output."""
    x = np.ascontiguousarray(x, np.float32)
    p = FftPlan(x.size, device)
    return freqs(x.size, rate)[x.size // 2:], p.exec_real(x)


class Stft:
    """Streaming Window(n) + Decimate(hop) + fft (adapters/mod.rs:270-303, 13-41).

    input_kind=CU8 takes raw rtl_tcp I/Q bytes (examples/live.rs windows rtl.listen()
    directly); output='db' yields f32 dB magnitudes (src/plot/complexseries.rs:90-92)."""

    def __init__(self, n: int, hop: int, device: int = 0, input_kind: int = _lib.C64,
                 output: str = "complex"):
        self.n, self.hop, self.device = int(n), int(hop), device
        self.input_kind, self.output = input_kind, output
        self._odt = np.float32 if output == "db" else np.complex64
        self._h = ctypes.c_void_p()
        check(lib().sdrgpu_stft_create(device, self.n, self.hop, ctypes.byref(self._h)),
              "sdrgpu_stft_create")
        check(lib().sdrgpu_stft_set_input_kind(self._h, input_kind), "sdrgpu_stft_set_input_kind")
        check(lib().sdrgpu_stft_set_output(self._h, _out_mode(output)), "sdrgpu_stft_set_output")

    def _as_in(self, x):
        if self.input_kind == _lib.CU8:
            return np.ascontiguousarray(x, np.uint8).reshape(-1)
        return np.ascontiguousarray(x, np.complex64)

    def _nsamp(self, x):
        return x.size // 2 if self.input_kind == _lib.CU8 else x.size

    def close(self):
        if self._h:
            lib().sdrgpu_stft_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().sdrgpu_stft_get_stream(self._h, ctypes.byref(s)), "get_stream")
        return s.value or 0

    def output_len(self, n_in: int) -> int:
        n = ctypes.c_size_t()
        check(lib().sdrgpu_stft_output_len(self._h, n_in, ctypes.byref(n)), "output_len")
        return n.value

    def process(self, x) -> np.ndarray:
        x = self._as_in(x)
        ns = self._nsamp(x)
        nf = self.output_len(ns)
        out = np.empty((max(nf, 1), self.n), self._odt)
        got = ctypes.c_size_t()
        check(lib().sdrgpu_stft_process(self._h, x.ctypes.data, ns, out.ctypes.data,
                                        nf, ctypes.byref(got)), "sdrgpu_stft_process")
        return out[:got.value]

    def process_async(self, in_ptr: int, n_in: int, out_ptr: int, cap_frames: int) -> int:
        """Pinned host blocks (device.PinnedBuffer), enqueued without waiting; returns the
        frame count.  Read the output after sync()."""
        got = ctypes.c_size_t()
        check(lib().sdrgpu_stft_process_async(self._h, in_ptr, n_in, out_ptr, cap_frames,
                                              ctypes.byref(got)), "sdrgpu_stft_process_async")
        return got.value

    def process_dev(self, d_in: int, n_in: int, d_out: int, cap_frames: int) -> int:
        got = ctypes.c_size_t()
        check(lib().sdrgpu_stft_process_dev(self._h, d_in, n_in, d_out, cap_frames,
                                            ctypes.byref(got)), "sdrgpu_stft_process_dev")
        return got.value

    def reset(self):
        check(lib().sdrgpu_stft_reset(self._h), "sdrgpu_stft_reset")

    def sync(self):
        check(lib().sdrgpu_stft_sync(self._h), "sdrgpu_stft_sync")
