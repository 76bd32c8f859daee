"""ctypes binding of include/sdrgpu.h (libsdrgpu.so, built in-tree for gfx950).

The product path is the HIP library only: if libsdrgpu.so is missing this module raises
on import -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_long, c_size_t, c_uint8, c_uint32, c_void_p

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_ROOT, "libsdrgpu.so")

OK = 0
ERR_INVALID = 1
ERR_NOMEM = 2
ERR_DEVICE = 3
ERR_NODEVICE = 4
ERR_UNSUPPORTED = 5
ERR_OUTPUT_CAP = 6
ERR_LAUNCH = 7

F32 = 0
C64 = 1
CU8 = 2   # FIR input: interleaved u8 I/Q from rtl_tcp, (v-128)/128 fused into the load

FIR_AUTO = 0
FIR_DIRECT = 1
FIR_OVERLAP_SAVE = 2
FIR_MATRIX = 3

# sdrgpu_fir_kernel: which kernel ran the last block (last_kernel())
FIR_KERNEL_NONE = 0
FIR_KERNEL_FP16 = 1
FIR_KERNEL_INT8 = 2
FIR_KERNEL_BF16X3 = 3
FIR_KERNEL_OVERLAP_SAVE = 4
FIR_KERNEL_DIRECT = 5
FIR_KERNEL_CU8_CONVERTED = 16

FFT_OUT_COMPLEX = 0
FFT_OUT_DB = 1

PLL_OUT_FILTER = 0
PLL_OUT_STEREO_DIFF = 1

DEBUG_ATAN2F = 0
DEBUG_SINCOSF = 1

BQ_IDENTITY = 0
BQ_LOWPASS = 1
BQ_HIGHPASS = 2
BQ_BANDPASS = 3
BQ_NOTCH = 4
BQ_LR = 5


class BiquadDesignC(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("freq", c_float), ("q", c_float)]


class PllParamsC(ctypes.Structure):
    _fields_ = [
        ("reference", c_float),
        ("gain", c_float),
        ("rate", c_float),
        ("loopf", BiquadDesignC),
        ("outputf", BiquadDesignC),
        ("lockf", BiquadDesignC),
    ]


class SdrGpuError(RuntimeError):
    """Non-zero sdrgpu status (mirrors resample::Error, reference src/resample.rs:151-270)."""

    def __init__(self, code: int, where: str = ""):
        self.code = code
        msg = lib().sdrgpu_strerror(code).decode() if _LIB is not None else str(code)
        super().__init__(f"{where}: sdrgpu error {code} ({msg})" if where else msg)


# (name, restype, argtypes) for every symbol in include/sdrgpu.h
_H = c_void_p
_PH = POINTER(c_void_p)
_PS = POINTER(c_size_t)
SIGNATURES = [
    ("sdrgpu_strerror", c_char_p, [c_int]),
    ("sdrgpu_abi_version", c_int, []),
    ("sdrgpu_device_count", c_int, [POINTER(c_int)]),
    # device memory / events
    ("sdrgpu_dev_alloc", c_int, [c_int, c_size_t, _PH]),
    ("sdrgpu_dev_free", c_int, [c_int, c_void_p]),
    ("sdrgpu_host_alloc", c_int, [c_int, c_size_t, _PH]),
    ("sdrgpu_host_free", c_int, [c_void_p]),
    ("sdrgpu_dev_copy", c_int, [c_int, c_void_p, c_void_p, c_size_t, c_int]),
    ("sdrgpu_dev_memset", c_int, [c_int, c_void_p, c_int, c_size_t]),
    ("sdrgpu_dev_synchronize", c_int, [c_int]),
    ("sdrgpu_event_create", c_int, [c_int, _PH]),
    ("sdrgpu_event_record", c_int, [c_void_p, c_void_p]),
    ("sdrgpu_event_synchronize", c_int, [c_void_p]),
    ("sdrgpu_event_elapsed_ms", c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    ("sdrgpu_event_destroy", c_int, [c_void_p]),
    # FIR
    ("sdrgpu_fir_create", c_int, [c_int, c_int, c_int, c_void_p, c_size_t, c_uint32, _PH]),
    ("sdrgpu_fir_set_algorithm", c_int, [_H, c_int]),
    ("sdrgpu_fir_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_fir_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_fir_output_len", c_int, [_H, c_size_t, _PS]),
    ("sdrgpu_fir_process", c_int, [_H, c_void_p, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_fir_process_dev", c_int, [_H, c_void_p, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_fir_process_async", c_int, [_H, c_void_p, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_fir_sync", c_int, [_H]),
    ("sdrgpu_fir_last_algorithm", c_int, [_H, POINTER(c_int)]),
    ("sdrgpu_fir_last_kernel", c_int, [_H, POINTER(c_int)]),
    ("sdrgpu_fir_reset", c_int, [_H]),
    ("sdrgpu_fir_clone", c_int, [_H, _PH]),
    ("sdrgpu_fir_destroy", None, [_H]),
    # FIR bank
    ("sdrgpu_firbank_create", c_int,
     [c_int, c_int, c_int, c_void_p, c_size_t, c_uint32, c_size_t, _PH]),
    ("sdrgpu_firbank_set_algorithm", c_int, [_H, c_int]),
    ("sdrgpu_firbank_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_firbank_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_firbank_output_len", c_int, [_H, c_size_t, _PS]),
    ("sdrgpu_firbank_process", c_int,
     [_H, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_firbank_process_dev", c_int,
     [_H, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_firbank_sync", c_int, [_H]),
    ("sdrgpu_firbank_last_algorithm", c_int, [_H, POINTER(c_int)]),
    ("sdrgpu_firbank_last_kernel", c_int, [_H, POINTER(c_int)]),
    ("sdrgpu_firbank_reset", c_int, [_H]),
    ("sdrgpu_firbank_clone", c_int, [_H, _PH]),
    ("sdrgpu_firbank_destroy", None, [_H]),
    # FFT
    ("sdrgpu_fft_plan", c_int, [c_int, c_size_t, _PH]),
    ("sdrgpu_fft_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_fft_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_fft_exec", c_int, [_H, c_void_p, c_void_p, c_size_t]),
    ("sdrgpu_fft_exec_dev", c_int, [_H, c_void_p, c_void_p, c_size_t]),
    ("sdrgpu_rfft_exec", c_int, [_H, c_void_p, c_void_p, c_size_t]),

    ("sdrgpu_rfft_exec_dev", c_int, [_H, c_void_p, c_void_p, c_size_t]),
    ("sdrgpu_fft_set_output", c_int, [_H, c_int]),
    ("sdrgpu_fft_sync", c_int, [_H]),
    ("sdrgpu_fft_destroy", None, [_H]),
    ("sdrgpu_fft_freqs", c_int, [c_size_t, c_float, c_void_p]),
    # STFT
    ("sdrgpu_stft_create", c_int, [c_int, c_size_t, c_size_t, _PH]),
    ("sdrgpu_stft_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_stft_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_stft_output_len", c_int, [_H, c_size_t, _PS]),
    ("sdrgpu_stft_process", c_int, [_H, c_void_p, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_stft_process_dev", c_int, [_H, c_void_p, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_stft_process_async", c_int, [_H, c_void_p, c_size_t, c_void_p, c_size_t, _PS]),
    ("sdrgpu_stft_set_input_kind", c_int, [_H, c_int]),
    ("sdrgpu_stft_set_output", c_int, [_H, c_int]),
    ("sdrgpu_stft_sync", c_int, [_H]),
    ("sdrgpu_stft_reset", c_int, [_H]),
    ("sdrgpu_stft_destroy", None, [_H]),
    # PLL
    ("sdrgpu_pll_create", c_int, [c_int, POINTER(PllParamsC), c_size_t, _PH]),
    ("sdrgpu_pll_set_output_mode", c_int, [_H, c_int]),
    ("sdrgpu_pll_set_input_kind", c_int, [_H, c_int]),
    ("sdrgpu_pll_set_time_parallel", c_int, [_H, c_long, c_long]),
    ("sdrgpu_pll_time_parallel_plan", c_int, [_H, c_size_t, POINTER(c_long), POINTER(c_long)]),
    ("sdrgpu_pll_last_time_parallel", c_int, [_H, POINTER(c_long), POINTER(c_long)]),
    ("sdrgpu_pll_set_phase_timing", c_int, [_H, c_int]),
    ("sdrgpu_pll_last_phase_ms", c_int, [_H, POINTER(c_float), POINTER(c_float), POINTER(c_float)]),
    ("sdrgpu_pll_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_pll_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_pll_process", c_int,
     [_H, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p, c_size_t]),
    ("sdrgpu_pll_process_dev", c_int,
     [_H, c_void_p, c_size_t, c_size_t, c_void_p, c_void_p, c_size_t]),
    ("sdrgpu_pll_process_async", c_int, [_H, c_void_p, c_size_t, c_void_p, c_void_p]),
    ("sdrgpu_pll_state", c_int, [_H, c_size_t, POINTER(c_float), POINTER(c_float)]),
    ("sdrgpu_pll_sync", c_int, [_H]),
    ("sdrgpu_pll_reset", c_int, [_H]),
    ("sdrgpu_pll_clone", c_int, [_H, _PH]),
    ("sdrgpu_pll_destroy", None, [_H]),
    ("sdrgpu_debug_libm", c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    # batched biquad
    ("sdrgpu_biquad_create", c_int, [c_int, c_int, POINTER(BiquadDesignC), c_float, c_size_t, _PH]),
    ("sdrgpu_biquad_coefs", c_int, [_H, POINTER(c_float)]),
    ("sdrgpu_biquad_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_biquad_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_biquad_process", c_int, [_H, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t]),
    ("sdrgpu_biquad_process_dev", c_int, [_H, c_void_p, c_size_t, c_size_t, c_void_p, c_size_t]),
    ("sdrgpu_biquad_set_time_parallel", c_int, [_H, c_long, c_long]),
    ("sdrgpu_biquad_time_parallel_plan", c_int, [_H, c_size_t, POINTER(c_long), POINTER(c_long)]),
    ("sdrgpu_biquad_last_time_parallel", c_int, [_H, POINTER(c_long), POINTER(c_long)]),
    ("sdrgpu_biquad_sync", c_int, [_H]),
    ("sdrgpu_biquad_reset", c_int, [_H]),
    ("sdrgpu_biquad_clone", c_int, [_H, _PH]),
    ("sdrgpu_biquad_destroy", None, [_H]),
    # sample-rate conversion (libsamplerate surface; returns libsamplerate codes)
    ("sdrgpu_src_new", c_void_p, [c_int, c_int, c_int, POINTER(c_int)]),
    ("sdrgpu_src_process", c_int, [_H, c_void_p]),
    ("sdrgpu_src_process_dev", c_int, [_H, c_void_p]),
    ("sdrgpu_src_sync", c_int, [_H]),
    ("sdrgpu_src_reset", c_int, [_H]),
    ("sdrgpu_src_clone", c_void_p, [_H, POINTER(c_int)]),
    ("sdrgpu_src_get_channels", c_int, [_H]),
    ("sdrgpu_src_set_ratio", c_int, [_H, ctypes.c_double]),
    ("sdrgpu_src_set_stream", c_int, [_H, c_void_p]),
    ("sdrgpu_src_get_stream", c_int, [_H, _PH]),
    ("sdrgpu_src_delete", c_void_p, [_H]),
    ("sdrgpu_src_strerror", c_char_p, [c_int]),
    ("sdrgpu_src_get_name", c_char_p, [c_int]),
    ("sdrgpu_src_get_description", c_char_p, [c_int]),
    ("sdrgpu_src_get_version", c_char_p, []),
    ("sdrgpu_src_sinc_table", c_int, [c_int, c_void_p, c_int, POINTER(c_int)]),
    # multi-GPU fan-out / gather (RCCL)
    ("sdrgpu_comm_unique_id", c_int, [c_void_p]),
    ("sdrgpu_comm_init", c_int, [c_int, c_int, c_int, c_void_p, _PH]),
    ("sdrgpu_comm_scatter", c_int, [_H, c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    ("sdrgpu_comm_gather", c_int, [_H, c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    ("sdrgpu_comm_scatterv", c_int, [_H, c_void_p, _PS, _PS, c_void_p, c_int, c_void_p]),
    ("sdrgpu_comm_gatherv", c_int, [_H, c_void_p, c_void_p, _PS, _PS, c_int, c_void_p]),
    ("sdrgpu_comm_barrier", c_int, [_H, c_void_p]),
    ("sdrgpu_comm_destroy", None, [_H]),
    ("sdrgpu_comm_plan_v", c_int, [c_int, c_int, c_int, c_int, _PS, _PS, c_void_p, c_int,
                                   POINTER(c_int)]),
]

_LIB = None


def lib() -> ctypes.CDLL:
    """Load libsdrgpu.so (fails loudly when the HIP extension was not built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build it with `make -C unnamed-rust-sdr_amd` "
                "(or __graft_entry__.build()); sdrgpu has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(code: int, where: str = "") -> None:
    if code != OK:
        raise SdrGpuError(code, where)


def device_count() -> int:
    n = c_int(0)
    check(lib().sdrgpu_device_count(ctypes.byref(n)), "device_count")
    return n.value


__all__ = [n for n in dir() if not n.startswith("__")]
_ = (c_uint8,)
