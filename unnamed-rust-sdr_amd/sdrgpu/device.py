"""Device buffers and HIP events through the sdrgpu C ABI (no torch GPU runtime needed).

torch ships its own HIP runtime (torch/lib/libamdhip64.so); libsdrgpu links the system
ROCm runtime.  Handles and pointers of one runtime are not valid in the other, so code
that drives sdrgpu allocates and times through these helpers instead of torch.cuda.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib

H2D, D2H, D2D = 0, 1, 2


class DeviceBuffer:
    """A device allocation of `nbytes` (typed view helpers for f32 / c64 samples)."""

    def __init__(self, nbytes: int, device: int = 0, dtype=np.complex64):
        self.device = device
        self.nbytes = int(nbytes)
        self.dtype = np.dtype(dtype)
        p = ctypes.c_void_p()
        check(lib().sdrgpu_dev_alloc(device, self.nbytes, ctypes.byref(p)), "sdrgpu_dev_alloc")
        self.ptr = p.value

    @classmethod
    def empty(cls, n: int, dtype=np.complex64, device: int = 0) -> "DeviceBuffer":
        return cls(n * np.dtype(dtype).itemsize, device, dtype)

    @classmethod
    def from_numpy(cls, a: np.ndarray, device: int = 0) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, device, a.dtype)
        b.upload(a)
        return b

    def __len__(self):
        return self.nbytes // self.dtype.itemsize

    def upload(self, a: np.ndarray, offset_bytes: int = 0):
        a = np.ascontiguousarray(a)
        assert offset_bytes + a.nbytes <= self.nbytes
        check(lib().sdrgpu_dev_copy(self.device, self.ptr + offset_bytes, a.ctypes.data,
                                    a.nbytes, H2D), "upload")

    def download(self, n: int = None, dtype=None, offset_bytes: int = 0) -> np.ndarray:
        dtype = np.dtype(dtype or self.dtype)
        if n is None:
            n = (self.nbytes - offset_bytes) // dtype.itemsize
        out = np.empty(n, dtype)
        assert offset_bytes + out.nbytes <= self.nbytes
        check(lib().sdrgpu_dev_copy(self.device, out.ctypes.data, self.ptr + offset_bytes,
                                    out.nbytes, D2H), "download")
        return out

    def copy_from(self, src: "DeviceBuffer", nbytes: int, dst_off: int = 0, src_off: int = 0):
        check(lib().sdrgpu_dev_copy(self.device, self.ptr + dst_off, src.ptr + src_off, nbytes,
                                    D2D), "copy_from")

    def fill_zero(self):
        check(lib().sdrgpu_dev_memset(self.device, self.ptr, 0, self.nbytes), "memset")

    def free(self):
        if self.ptr:
            lib().sdrgpu_dev_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host memory (sdrgpu_host_alloc) viewed as a numpy array; the buffer type
    the *_async entry points stream from/to without blocking."""

    def __init__(self, n: int, dtype=np.complex64, device: int = 0):
        self.dtype = np.dtype(dtype)
        self.n = int(n)
        p = ctypes.c_void_p()
        check(lib().sdrgpu_host_alloc(device, max(1, self.n * self.dtype.itemsize),
                                      ctypes.byref(p)), "sdrgpu_host_alloc")
        self.ptr = p.value
        buf = (ctypes.c_char * (self.n * self.dtype.itemsize)).from_address(self.ptr)
        self.array = np.frombuffer(buf, dtype=self.dtype, count=self.n)

    def free(self):
        if getattr(self, "ptr", None):
            self.array = None
            lib().sdrgpu_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Event:
    def __init__(self, device: int = 0):
        p = ctypes.c_void_p()
        check(lib().sdrgpu_event_create(device, ctypes.byref(p)), "sdrgpu_event_create")
        self.ev = p.value

    def record(self, stream: int):
        check(lib().sdrgpu_event_record(self.ev, stream), "sdrgpu_event_record")

    def synchronize(self):
        check(lib().sdrgpu_event_synchronize(self.ev), "sdrgpu_event_synchronize")

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        check(lib().sdrgpu_event_elapsed_ms(self.ev, end.ev, ctypes.byref(ms)), "elapsed")
        return ms.value

    def __del__(self):
        try:
            if self.ev:
                lib().sdrgpu_event_destroy(self.ev)
                self.ev = None
        except Exception:
            pass


def synchronize(device: int = 0):
    check(lib().sdrgpu_dev_synchronize(device), "sdrgpu_dev_synchronize")
