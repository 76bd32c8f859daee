"""Host-side mirror of the reference `resample` module (src/resample.rs) over sdrgpu.

`SampleRate` keeps the reference's surface -- new(ConverterType), process(ratio, input,
out_cap) -> (input_used, output), reset(), try_clone(), channels(), set_ratio(), and the
Error enum with libsamplerate's codes (src/resample.rs:151-270) -- on top of the
`sdrgpu_src_*` C ABI (include/sdrgpu.h), which restates libsamplerate's converters on the
GPU: zero-order hold and linear bit-exactly; the sinc converters with libsamplerate 0.2's
src_sinc.c algorithm over this library's own Kaiser-windowed sinc tables (libsamplerate's
coefficient headers are not available, so sinc outputs are not libsamplerate's; DESIGN.md
3.7).

Frames: an input array of shape (n, channels) float32, or 1-D float32 (channels = 1) /
complex64 (channels = 2, num::Complex<f32> as [f32; 2], src/resample.rs:272-278).
"""
from __future__ import annotations

import ctypes
import enum
from ctypes import c_double, c_int, c_long, c_void_p

import numpy as np

from ._lib import lib


class ConverterType(enum.IntEnum):
    """resample::ConverterType (src/resample.rs:112-149), libsamplerate ids."""
    SincBestQuality = 0
    SincMediumQuality = 1
    SincFastest = 2
    ZeroOrderHold = 3
    Linear = 4

    def name_(self) -> str:
        return lib().sdrgpu_src_get_name(int(self)).decode()

    def description(self) -> str:
        return lib().sdrgpu_src_get_description(int(self)).decode()


class Error(RuntimeError):
    """resample::Error: libsamplerate's error code and its description (:151-270)."""
    NAMES = {1: "MallocFailed", 2: "BadState", 3: "BadData", 4: "BadDataPtr", 5: "NoPrivate",
             6: "BadSrcRatio", 7: "BadProcPtr", 8: "ShiftBits", 9: "FilterLen",
             10: "BadConverter", 11: "BadChannelCount", 12: "SincBadBufferLen",
             13: "SizeIncompatibility", 14: "BadPrivPtr", 15: "BadSincState",
             16: "DataOverlap", 17: "BadCallback", 18: "BadMode", 19: "NullCallback",
             20: "NoVariableRatio", 21: "SincPrepareDataBadLen", 22: "BadInternalState"}

    def __init__(self, code: int):
        self.code = code
        self.kind = self.NAMES.get(code, f"Unknown({code})")
        d = lib().sdrgpu_src_strerror(code)
        super().__init__(f"{self.kind}: {d.decode() if d else 'unknown error'}")

    @staticmethod
    def result(code: int):
        if code:
            raise Error(code)


class SrcData(ctypes.Structure):
    """libsamplerate SRC_DATA (sdrgpu_src_data)."""
    _fields_ = [("data_in", c_void_p), ("data_out", c_void_p), ("input_frames", c_long),
                ("output_frames", c_long), ("input_frames_used", c_long),
                ("output_frames_gen", c_long), ("end_of_input", c_int),
                ("src_ratio", c_double)]


_EMPTY = np.zeros(1, np.float32)


def sinc_table(typ: ConverterType):
    """(coefficients f32, increment) of a sinc converter's table (sdrgpu_src_sinc_table)."""
    inc = c_int(0)
    n = lib().sdrgpu_src_sinc_table(int(typ), None, 0, ctypes.byref(inc))
    if n < 0:
        raise Error(10)
    out = np.empty(n, np.float32)
    lib().sdrgpu_src_sinc_table(int(typ), out.ctypes.data, n, ctypes.byref(inc))
    return out, inc.value


def version() -> str:
    """resample::version (src/resample.rs:3-8)."""
    return lib().sdrgpu_src_get_version().decode()


def _frames(x, channels):
    x = np.asarray(x)
    if np.iscomplexobj(x):
        x = np.ascontiguousarray(x, np.complex64).view(np.float32)
    x = np.ascontiguousarray(x, np.float32)
    if x.size % channels:
        raise ValueError(f"{x.size} floats is not a whole number of {channels}-channel frames")
    return x.reshape(-1, channels)


class SampleRate:
    """resample::SampleRate<A> (src/resample.rs:10-110) on one GPU."""

    def __init__(self, typ: ConverterType, channels: int = 1, device: int = 0, _h=None):
        self.device = device
        self._ch = channels
        if _h is not None:
            self.h = _h
            return
        err = c_int(0)
        self.h = lib().sdrgpu_src_new(device, int(typ), channels, ctypes.byref(err))
        if not self.h:
            raise Error(err.value or 2)

    def __del__(self):
        if getattr(self, "h", None):
            lib().sdrgpu_src_delete(self.h)
            self.h = None

    def process(self, ratio: float, input, out_cap: int):
        """SampleRate::process (:46-67): returns (input_frames_used, output frames)."""
        x = _frames(input, self._ch)
        out = np.empty((max(int(out_cap), 1), self._ch), np.float32)
        # an empty Rust slice has a non-NULL pointer, so src_process sees end_of_input
        # with data_in set and the sinc converters flush (src/resample.rs:47-56)
        if not x.shape[0]:
            x = np.zeros((1, self._ch), np.float32)[:0]
        d = SrcData(x.ctypes.data or _EMPTY.ctypes.data, out.ctypes.data, x.shape[0],
                    int(out_cap), 0, 0, 1 if x.shape[0] == 0 else 0, float(ratio))
        Error.result(lib().sdrgpu_src_process(self.h, ctypes.byref(d)))
        return d.input_frames_used, out[:d.output_frames_gen].copy()

    def process_dev(self, ratio: float, d_in: int, in_frames: int, d_out: int,
                    out_frames: int):
        """Device-pointer variant: counts return at once, the conversion is enqueued."""
        d = SrcData(d_in or _EMPTY.ctypes.data, d_out or None, in_frames, out_frames, 0, 0,
                    1 if in_frames == 0 else 0, float(ratio))
        Error.result(lib().sdrgpu_src_process_dev(self.h, ctypes.byref(d)))
        return d.input_frames_used, d.output_frames_gen

    def stream(self) -> int:
        p = c_void_p()
        Error.result(lib().sdrgpu_src_get_stream(self.h, ctypes.byref(p)))
        return p.value or 0

    def sync(self):
        Error.result(lib().sdrgpu_src_sync(self.h))

    def reset(self):
        Error.result(lib().sdrgpu_src_reset(self.h))

    def try_clone(self) -> "SampleRate":
        err = c_int(0)
        h = lib().sdrgpu_src_clone(self.h, ctypes.byref(err))
        if not h:
            raise Error(err.value or 2)
        return SampleRate(ConverterType.Linear, self._ch, self.device, _h=h)

    clone = try_clone

    def channels(self) -> int:
        return lib().sdrgpu_src_get_channels(self.h)

    def set_ratio(self, ratio: float):
        Error.result(lib().sdrgpu_src_set_ratio(self.h, float(ratio)))
