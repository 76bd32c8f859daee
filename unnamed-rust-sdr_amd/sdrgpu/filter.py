"""Host-side mirror of the reference `filter` module over the sdrgpu C ABI.

Reference interface (agrif/unnamed-rust-sdr):
  trait Filter<A>        { fn apply(&mut self, A) -> Output }      src/filter/mod.rs:23-26
  trait FilterDesign<A>  { fn design(self, rate) -> Filter;
                           fn design_for(self, &signal) }          src/filter/mod.rs:28-39
  Fir / Vec<C> / &[C] designs                                       src/filter/fir.rs:36-58
  BiquadD::{LowPass,HighPass,BandPass,Notch,Lr}                     src/filter/biquad.rs:63-155
  Identity                                                          src/filter/simple.rs:3-19
  PllDesign::new(reference, gain, loop, output, lock)               src/filter/pll.rs:25-37

Names and argument meaning follow the reference.  Designs are plain values; `design(rate)`
returns a GPU-backed filter handle.  Because a per-sample FFI call is infeasible, handles
process BLOCKS (`process`) -- `apply` exists for API parity and is a one-sample block.
State carries across blocks, so any block partition yields the reference's sample-by-
sample result.  Handles are Send-not-Sync like the reference filters.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence, Union

import numpy as np

from . import _lib
from ._lib import C64, CU8, F32, check, lib


def _kind_of(arr: np.ndarray) -> int:
    if np.iscomplexobj(arr):
        return C64
    return F32


def _as_c(arr, kind: int) -> np.ndarray:
    if kind == C64:
        return np.ascontiguousarray(arr, dtype=np.complex64)
    if kind == CU8:
        # rtl_tcp byte stream: interleaved I/Q bytes, (..., 2n) or (..., n, 2)
        return np.ascontiguousarray(arr, dtype=np.uint8)
    return np.ascontiguousarray(arr, dtype=np.float32)


def _nsamp(x: np.ndarray, kind: int) -> int:
    """samples along the last stream axis (CU8: 2 bytes per sample)."""
    if kind != CU8:
        return x.shape[-1] if x.ndim else 1
    if x.ndim >= 2 and x.shape[-1] == 2:
        return x.shape[-2]
    return x.shape[-1] // 2


def _np_dtype(kind: int):
    return np.complex64 if kind in (C64, CU8) else np.float32


# ------------------------------------------------------------------------------ FIR
class Fir:
    """FilterDesign for FIR taps: `Fir::new(coef)` / `Vec<C>` / `&[C]` (fir.rs:12-58).

    `decim` (default 1) fuses the reference's `.decimate(rate)` adapter that usually
    follows (signal/adapters/mod.rs:13-41): only outputs at stream indices D-1, 2D-1, ...
    are produced.  `sample_kind` selects f32 or Complex<f32> samples (the reference infers
    A from the signal; design_for() does the same here)."""

    def __init__(self, coef: Union[Sequence, np.ndarray], decim: int = 1,
                 sample_kind: Optional[int] = None, device: int = 0,
                 algorithm: int = _lib.FIR_AUTO):
        coef = np.asarray(coef)
        if coef.ndim != 1 or coef.size == 0:
            raise _lib.SdrGpuError(_lib.ERR_INVALID, "Fir: taps must be a non-empty 1-D array")
        self.tap_kind = _kind_of(coef)
        self.coef = _as_c(coef, self.tap_kind)
        self.decim = int(decim)
        self.sample_kind = sample_kind
        self.device = device
        self.algorithm = algorithm

    def with_decim(self, decim: int) -> "Fir":
        return Fir(self.coef, decim, self.sample_kind, self.device, self.algorithm)

    def design(self, rate: float = 0.0, sample_kind: Optional[int] = None) -> "FirFilter":
        """FilterDesign::design -- rate is unused for FIR (fir.rs:39)."""
        sk = sample_kind if sample_kind is not None else self.sample_kind
        if sk is None:
            sk = C64 if self.tap_kind == C64 else F32
        return FirFilter(self.coef, sk, self.decim, self.device, self.algorithm)

    def design_for(self, signal) -> "FirFilter":
        return self.design(signal.rate(), getattr(signal, "sample_kind", None))


class FirFilter:
    """GPU Fir<C, A> handle (fir.rs:6-32) with optional fused decimation."""

    def __init__(self, coef: np.ndarray, sample_kind: int, decim: int = 1, device: int = 0,
                 algorithm: int = _lib.FIR_AUTO, _handle=None):
        self.sample_kind = sample_kind
        self.tap_kind = _kind_of(coef)
        self.coef = coef
        self.decim = decim
        self.device = device
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            check(lib().sdrgpu_fir_create(device, sample_kind, self.tap_kind,
                                          coef.ctypes.data, coef.size, decim,
                                          ctypes.byref(self._h)), "sdrgpu_fir_create")
        if algorithm != _lib.FIR_AUTO:
            self.set_algorithm(algorithm)

    # -- handle management (SampleRate-style, resample.rs:32-110) --
    def close(self):
        if self._h:
            lib().sdrgpu_fir_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def clone(self) -> "FirFilter":
        h = ctypes.c_void_p()
        check(lib().sdrgpu_fir_clone(self._h, ctypes.byref(h)), "sdrgpu_fir_clone")
        return FirFilter(self.coef, self.sample_kind, self.decim, self.device, _handle=h)

    def reset(self):
        check(lib().sdrgpu_fir_reset(self._h), "sdrgpu_fir_reset")

    def set_algorithm(self, algo: int):
        check(lib().sdrgpu_fir_set_algorithm(self._h, algo), "sdrgpu_fir_set_algorithm")

    def set_stream(self, stream_ptr: Optional[int]):
        check(lib().sdrgpu_fir_set_stream(self._h, stream_ptr), "sdrgpu_fir_set_stream")

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().sdrgpu_fir_get_stream(self._h, ctypes.byref(s)), "sdrgpu_fir_get_stream")
        return s.value or 0

    def output_len(self, n_in: int) -> int:
        n = ctypes.c_size_t()
        check(lib().sdrgpu_fir_output_len(self._h, n_in, ctypes.byref(n)), "output_len")
        return n.value

    # -- processing --
    def process(self, x) -> np.ndarray:
        """Filter one block of host samples; returns the (kept) outputs."""
        x = _as_c(x, self.sample_kind)
        n_in = _nsamp(x.reshape(-1), self.sample_kind)
        n_out = self.output_len(n_in)
        out = np.empty(max(n_out, 1), dtype=_np_dtype(self.sample_kind))
        got = ctypes.c_size_t()
        check(lib().sdrgpu_fir_process(self._h, x.ctypes.data, n_in, out.ctypes.data,
                                       out.size, ctypes.byref(got)), "sdrgpu_fir_process")
        return out[:got.value]

    def apply(self, value):
        """Filter::apply for one sample (fir.rs:23-32).  Returns None when decimation
        drops the sample (the Decimate adapter would skip it)."""
        y = self.process(np.asarray([value]))
        return y[0] if y.size else None

    def process_async(self, in_ptr: int, n_in: int, out_ptr: int, out_cap: int) -> int:
        """Host pointers (pinned: device.PinnedBuffer), enqueued without waiting; returns
        n_out.  Read the output after sync()."""
        got = ctypes.c_size_t()
        check(lib().sdrgpu_fir_process_async(self._h, in_ptr, n_in, out_ptr, out_cap,
                                             ctypes.byref(got)), "sdrgpu_fir_process_async")
        return got.value

    def process_dev(self, d_in_ptr: int, n_in: int, d_out_ptr: int, out_cap: int) -> int:
        """Enqueue on the handle's stream with device pointers; returns n_out."""
        got = ctypes.c_size_t()
        check(lib().sdrgpu_fir_process_dev(self._h, d_in_ptr, n_in, d_out_ptr, out_cap,
                                           ctypes.byref(got)), "sdrgpu_fir_process_dev")
        return got.value

    def sync(self):
        check(lib().sdrgpu_fir_sync(self._h), "sdrgpu_fir_sync")

    def last_algorithm(self) -> int:
        """FIR_DIRECT / FIR_OVERLAP_SAVE / FIR_MATRIX: the path of the last block."""
        a = ctypes.c_int()
        check(lib().sdrgpu_fir_last_algorithm(self._h, ctypes.byref(a)), "last_algorithm")
        return a.value

    def last_kernel(self) -> int:
        """FIR_KERNEL_*: the kernel of the last block (| FIR_KERNEL_CU8_CONVERTED when u8
        input was converted to c64 by its own launch first)."""
        a = ctypes.c_int()
        check(lib().sdrgpu_fir_last_kernel(self._h, ctypes.byref(a)), "last_kernel")
        return a.value


class FirBank:
    """nch independent Fir<C,A> (fir.rs:6-32) sharing taps; channel-major blocks."""

    def __init__(self, coef, nch: int, sample_kind: int = C64, decim: int = 1,
                 device: int = 0, algorithm: int = _lib.FIR_AUTO, _handle=None):
        coef = np.asarray(coef)
        self.tap_kind = _kind_of(coef)
        self.coef = _as_c(coef, self.tap_kind)
        self.nch = nch
        self.sample_kind = sample_kind
        self.decim = decim
        self.device = device
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            check(lib().sdrgpu_firbank_create(device, sample_kind, self.tap_kind,
                                              self.coef.ctypes.data, self.coef.size, decim,
                                              nch, ctypes.byref(self._h)),
                  "sdrgpu_firbank_create")
        if algorithm != _lib.FIR_AUTO:
            self.set_algorithm(algorithm)

    def close(self):
        if self._h:
            lib().sdrgpu_firbank_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def clone(self) -> "FirBank":
        h = ctypes.c_void_p()
        check(lib().sdrgpu_firbank_clone(self._h, ctypes.byref(h)), "sdrgpu_firbank_clone")
        return FirBank(self.coef, self.nch, self.sample_kind, self.decim, self.device,
                       _handle=h)

    def reset(self):
        check(lib().sdrgpu_firbank_reset(self._h), "sdrgpu_firbank_reset")

    def set_algorithm(self, algo: int):
        check(lib().sdrgpu_firbank_set_algorithm(self._h, algo), "set_algorithm")

    def set_stream(self, stream_ptr: Optional[int]):
        check(lib().sdrgpu_firbank_set_stream(self._h, stream_ptr), "set_stream")

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().sdrgpu_firbank_get_stream(self._h, ctypes.byref(s)), "get_stream")
        return s.value or 0

    def output_len(self, n_in: int) -> int:
        n = ctypes.c_size_t()
        check(lib().sdrgpu_firbank_output_len(self._h, n_in, ctypes.byref(n)), "output_len")
        return n.value

    def process(self, x) -> np.ndarray:
        """x: (nch, n) host array -> (nch, n_out)."""
        x = _as_c(x, self.sample_kind)
        if x.ndim == 3 and self.sample_kind == CU8:
            x = x.reshape(x.shape[0], -1)
        if x.ndim != 2 or x.shape[0] != self.nch:
            raise _lib.SdrGpuError(_lib.ERR_INVALID, "FirBank.process: shape must be (nch, n)")
        n_in = _nsamp(x, self.sample_kind)
        n_out = self.output_len(n_in)
        out = np.empty((self.nch, max(n_out, 1)), dtype=_np_dtype(self.sample_kind))
        got = ctypes.c_size_t()
        check(lib().sdrgpu_firbank_process(self._h, x.ctypes.data, n_in, n_in,
                                           out.ctypes.data, out.shape[1], ctypes.byref(got)),
              "sdrgpu_firbank_process")
        return out[:, :got.value]

    def process_dev(self, d_in_ptr: int, ld_in: int, n_in: int, d_out_ptr: int,
                    ld_out: int) -> int:
        got = ctypes.c_size_t()
        check(lib().sdrgpu_firbank_process_dev(self._h, d_in_ptr, ld_in, n_in, d_out_ptr,
                                               ld_out, ctypes.byref(got)),
              "sdrgpu_firbank_process_dev")
        return got.value

    def sync(self):
        check(lib().sdrgpu_firbank_sync(self._h), "sdrgpu_firbank_sync")

    def last_algorithm(self) -> int:
        a = ctypes.c_int()
        check(lib().sdrgpu_firbank_last_algorithm(self._h, ctypes.byref(a)), "last_algorithm")
        return a.value

    def last_kernel(self) -> int:
        a = ctypes.c_int()
        check(lib().sdrgpu_firbank_last_kernel(self._h, ctypes.byref(a)), "last_kernel")
        return a.value


# --------------------------------------------------------------------------- Biquad
@dataclass(frozen=True)
class BiquadD:
    """BiquadD enum (biquad.rs:63-71).  Construct with the class helpers below."""
    kind: int
    freq: float
    q: float = 0.0

    @staticmethod
    def LowPass(freq: float, q: float) -> "BiquadD":
        return BiquadD(_lib.BQ_LOWPASS, freq, q)

    @staticmethod
    def HighPass(freq: float, q: float) -> "BiquadD":
        return BiquadD(_lib.BQ_HIGHPASS, freq, q)

    @staticmethod
    def BandPass(freq: float, q: float) -> "BiquadD":
        return BiquadD(_lib.BQ_BANDPASS, freq, q)

    @staticmethod
    def Notch(freq: float, q: float) -> "BiquadD":
        return BiquadD(_lib.BQ_NOTCH, freq, q)

    @staticmethod
    def Lr(decayrate: float) -> "BiquadD":
        return BiquadD(_lib.BQ_LR, decayrate, 0.0)

    def to_c(self) -> _lib.BiquadDesignC:
        return _lib.BiquadDesignC(self.kind, self.freq, self.q)

    def design(self, rate: float, sample_kind: int = F32, nch: int = 1,
               device: int = 0) -> "Biquad":
        """FilterDesign for BiquadD (biquad.rs:83-155): nch Biquad<C, f32> filters."""
        return Biquad(self.to_c(), rate, sample_kind, nch, device)


class _IdentityType:
    """filter::Identity (simple.rs:3-19)."""
    kind = _lib.BQ_IDENTITY
    freq = 0.0
    q = 0.0

    def to_c(self) -> _lib.BiquadDesignC:
        return _lib.BiquadDesignC(_lib.BQ_IDENTITY, 0.0, 0.0)

    def design(self, rate: float, sample_kind: int = F32, nch: int = 1,
               device: int = 0) -> "Biquad":
        return Biquad(self.to_c(), rate, sample_kind, nch, device)

    def __repr__(self):
        return "Identity"


Identity = _IdentityType()


# ------------------------------------------------------------------------------ PLL
class Biquad:
    """nch independent Biquad<C, f32> (biquad.rs:4-56) on the GPU, bit-identical outputs;
    `filter.Identity.design(...)` gives the pass-through (simple.rs:3-19)."""

    def __init__(self, design_c, rate: float, sample_kind: int = F32, nch: int = 1,
                 device: int = 0, _handle=None):
        self.design_c, self.rate, self.sample_kind = design_c, rate, sample_kind
        self.nch, self.device = nch, device
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            check(lib().sdrgpu_biquad_create(device, sample_kind, ctypes.byref(design_c), rate,
                                             nch, ctypes.byref(self._h)), "sdrgpu_biquad_create")

    def close(self):
        if self._h:
            lib().sdrgpu_biquad_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def coefs(self) -> np.ndarray:
        c = (ctypes.c_float * 5)()
        check(lib().sdrgpu_biquad_coefs(self._h, c), "sdrgpu_biquad_coefs")
        return np.array(c[:], dtype=np.float32)

    def clone(self) -> "Biquad":
        h = ctypes.c_void_p()
        check(lib().sdrgpu_biquad_clone(self._h, ctypes.byref(h)), "sdrgpu_biquad_clone")
        return Biquad(self.design_c, self.rate, self.sample_kind, self.nch, self.device,
                      _handle=h)

    def reset(self):
        check(lib().sdrgpu_biquad_reset(self._h), "sdrgpu_biquad_reset")

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().sdrgpu_biquad_get_stream(self._h, ctypes.byref(s)), "get_stream")
        return s.value or 0

    def process(self, x) -> np.ndarray:
        """x: (n,) for one channel or (nch, n) -> same shape, filtered."""
        x = _as_c(x, self.sample_kind)
        one = x.ndim == 1
        x2 = x.reshape(1, -1) if one else x
        if x2.shape[0] != self.nch:
            raise _lib.SdrGpuError(_lib.ERR_INVALID, "Biquad.process: shape must be (nch, n)")
        n = x2.shape[1]
        out = np.empty_like(x2)
        check(lib().sdrgpu_biquad_process(self._h, x2.ctypes.data, n, n, out.ctypes.data, n),
              "sdrgpu_biquad_process")
        return out[0] if one else out

    def apply(self, value):
        """Filter::apply for one sample (biquad.rs:42-56)."""
        return self.process(np.asarray([value]))[0]

    def process_dev(self, d_in, ld_in, n, d_out, ld_out):
        check(lib().sdrgpu_biquad_process_dev(self._h, d_in, ld_in, n, d_out, ld_out),
              "sdrgpu_biquad_process_dev")

    def set_time_parallel(self, seg: int = 0, warm: int = 0):
        """Segments of `seg` samples with `warm` samples of warm-up (0, 0: automatic; seg < 0:
        always serial); outputs identical to the serial recurrence."""
        check(lib().sdrgpu_biquad_set_time_parallel(self._h, seg, warm), "set_time_parallel")

    def time_parallel_plan(self, n: int):
        s, w = ctypes.c_long(), ctypes.c_long()
        check(lib().sdrgpu_biquad_time_parallel_plan(self._h, n, ctypes.byref(s), ctypes.byref(w)),
              "time_parallel_plan")
        return s.value, w.value

    def last_time_parallel(self):
        s, r = ctypes.c_long(), ctypes.c_long()
        check(lib().sdrgpu_biquad_last_time_parallel(self._h, ctypes.byref(s), ctypes.byref(r)),
              "last_time_parallel")
        return s.value, r.value

    def sync(self):
        check(lib().sdrgpu_biquad_sync(self._h), "sdrgpu_biquad_sync")


class PllDesign:
    """PllDesign::new(reference, gain, loopfilter, outputfilter, lockfilter)
    (pll.rs:25-37).  design(rate) -> Pll over `nch` independent channels."""

    def __init__(self, reference: float, gain: float, loopfilter, outputfilter, lockfilter):
        self.reference = reference
        self.gain = gain
        self.loopfilter = loopfilter
        self.outputfilter = outputfilter
        self.lockfilter = lockfilter

    def params(self, rate: float) -> _lib.PllParamsC:
        return _lib.PllParamsC(self.reference, self.gain, rate, self.loopfilter.to_c(),
                               self.outputfilter.to_c(), self.lockfilter.to_c())

    def design(self, rate: float, nch: int = 1, device: int = 0) -> "Pll":
        return Pll(self.params(rate), nch, device)


class Pll:
    """GPU Pll (pll.rs:12-22, 70-85), one per channel.  process() returns
    (output, locked): output = Some(v) -> v, None -> 0.0 (main.rs:49)."""

    def __init__(self, params: _lib.PllParamsC, nch: int = 1, device: int = 0, _handle=None):
        self.params = params
        self.nch = nch
        self.device = device
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            check(lib().sdrgpu_pll_create(device, ctypes.byref(params), nch,
                                          ctypes.byref(self._h)), "sdrgpu_pll_create")

    def close(self):
        if self._h:
            lib().sdrgpu_pll_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def clone(self) -> "Pll":
        h = ctypes.c_void_p()
        check(lib().sdrgpu_pll_clone(self._h, ctypes.byref(h)), "sdrgpu_pll_clone")
        return Pll(self.params, self.nch, self.device, _handle=h)

    def reset(self):
        check(lib().sdrgpu_pll_reset(self._h), "sdrgpu_pll_reset")

    def set_input_kind(self, kind: int):
        """_lib.C64 (default) or _lib.CU8 (raw rtl_tcp I/Q bytes) for process_dev /
        process_async (process / process_u8 set it themselves)."""
        check(lib().sdrgpu_pll_set_input_kind(self._h, kind), "sdrgpu_pll_set_input_kind")

    def set_output_mode(self, mode: int):
        """_lib.PLL_OUT_FILTER (Pll::apply's output) or _lib.PLL_OUT_STEREO_DIFF."""
        check(lib().sdrgpu_pll_set_output_mode(self._h, mode), "sdrgpu_pll_set_output_mode")

    def stereo(self, v):
        """src/main.rs:56-69 with this PLL as `pllpilot`: real audio v (nch, n) or (n,) ->
        (mono, diff, locked); mono = v * 0.5, diff = (v / value.powi(2)).re * 0.5 when the
        pilot is locked else 0.0."""
        v = np.ascontiguousarray(v, np.float32)
        self.set_output_mode(_lib.PLL_OUT_STEREO_DIFF)
        try:
            diff, locked = self.process(v.astype(np.complex64))  # Complex::new(v, 0.0)
        finally:
            self.set_output_mode(_lib.PLL_OUT_FILTER)
        return v * np.float32(0.5), diff, locked

    def set_time_parallel(self, seg: int = 0, warm: int = 0):
        """Time-parallel blocks (bit-identical results): seg = 0 automatic, < 0 off (one serial
        pass), > 0 a forced segment length; warm = warm-up samples (0: 16384)."""
        check(lib().sdrgpu_pll_set_time_parallel(self._h, seg, warm), "sdrgpu_pll_set_time_parallel")

    def last_time_parallel(self):
        """(segments, segments recomputed) of the most recent block (0, 0 when serial)."""
        a, b = ctypes.c_long(), ctypes.c_long()
        check(lib().sdrgpu_pll_last_time_parallel(self._h, ctypes.byref(a), ctypes.byref(b)),
              "sdrgpu_pll_last_time_parallel")
        return a.value, b.value

    def set_phase_timing(self, on: bool = True):
        """Record events around the three kernels of time-parallel blocks (measurement aid)."""
        check(lib().sdrgpu_pll_set_phase_timing(self._h, 1 if on else 0), "sdrgpu_pll_set_phase_timing")

    def last_phase_ms(self):
        """(pass 1, re-run pass, walk) ms of the most recent block (zeros when serial)."""
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        check(lib().sdrgpu_pll_last_phase_ms(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
              "sdrgpu_pll_last_phase_ms")
        return a.value, b.value, c.value

    def time_parallel_plan(self, n: int):
        """(segment length or 0 for one serial pass, warm-up) for a block of n samples."""
        seg, warm = ctypes.c_long(), ctypes.c_long()
        check(lib().sdrgpu_pll_time_parallel_plan(self._h, n, ctypes.byref(seg), ctypes.byref(warm)),
              "sdrgpu_pll_time_parallel_plan")
        return seg.value, warm.value

    def set_stream(self, stream_ptr):
        check(lib().sdrgpu_pll_set_stream(self._h, stream_ptr), "sdrgpu_pll_set_stream")

    def stream(self) -> int:
        s = ctypes.c_void_p()
        check(lib().sdrgpu_pll_get_stream(self._h, ctypes.byref(s)), "sdrgpu_pll_get_stream")
        return s.value or 0

    def process_u8(self, iq):
        """rtl_tcp bytes: iq (nch, 2n) or (2n,) uint8 interleaved I/Q -> (out, locked)."""
        iq = np.ascontiguousarray(iq, dtype=np.uint8)
        squeeze = iq.ndim == 1
        if squeeze:
            iq = iq[None, :]
        n = iq.shape[1] // 2
        out = np.empty((self.nch, max(n, 1)), dtype=np.float32)
        locked = np.empty((self.nch, max(n, 1)), dtype=np.uint8)
        check(lib().sdrgpu_pll_set_input_kind(self._h, CU8), "sdrgpu_pll_set_input_kind")
        try:
            check(lib().sdrgpu_pll_process(self._h, iq.ctypes.data, n, n, out.ctypes.data,
                                           locked.ctypes.data, out.shape[1]), "sdrgpu_pll_process")
        finally:
            check(lib().sdrgpu_pll_set_input_kind(self._h, C64), "sdrgpu_pll_set_input_kind")
        out, locked = out[:, :n], locked[:, :n]
        return (out[0], locked[0]) if squeeze else (out, locked)

    def process(self, x):
        """x: (nch, n) or (n,) complex -> (out float32, locked uint8) of the same shape."""
        x = np.ascontiguousarray(x, dtype=np.complex64)
        squeeze = x.ndim == 1
        if squeeze:
            x = x[None, :]
        if x.shape[0] != self.nch:
            raise _lib.SdrGpuError(_lib.ERR_INVALID, "Pll.process: expected nch rows")
        n = x.shape[1]
        out = np.empty((self.nch, max(n, 1)), dtype=np.float32)
        locked = np.empty((self.nch, max(n, 1)), dtype=np.uint8)
        check(lib().sdrgpu_pll_process(self._h, x.ctypes.data, n, n, out.ctypes.data,
                                       locked.ctypes.data, out.shape[1]), "sdrgpu_pll_process")
        out, locked = out[:, :n], locked[:, :n]
        return (out[0], locked[0]) if squeeze else (out, locked)

    def apply(self, value):
        """Filter::apply (pll.rs:70-85): Some(output) or None."""
        o, l = self.process(np.asarray([value], dtype=np.complex64))
        return float(o[0]) if l[0] else None

    def process_async(self, in_ptr: int, n: int, out_ptr: int, locked_ptr: int):
        """Pinned host blocks of nch x n samples (dense), enqueued without waiting; read the
        outputs after sync()."""
        check(lib().sdrgpu_pll_process_async(self._h, in_ptr, n, out_ptr, locked_ptr),
              "sdrgpu_pll_process_async")

    def process_dev(self, d_in, ld_in, n, d_out, d_locked, ld_out):
        check(lib().sdrgpu_pll_process_dev(self._h, d_in, ld_in, n, d_out, d_locked, ld_out),
              "sdrgpu_pll_process_dev")

    def state(self, ch: int = 0):
        """Public fields Pll::nphase, Pll::value (pll.rs:20-21)."""
        nph = ctypes.c_float()
        val = (ctypes.c_float * 2)()
        check(lib().sdrgpu_pll_state(self._h, ch, ctypes.byref(nph), val), "sdrgpu_pll_state")
        return nph.value, complex(val[0], val[1])

    def sync(self):
        check(lib().sdrgpu_pll_sync(self._h), "sdrgpu_pll_sync")
