"""CPU tests of the C-ABI boundary: the library loads, exports every declared symbol,
and rejects bad arguments without touching a GPU (no compute calls here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sdrgpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sdrgpu_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_api():
    names = declared_functions()
    for n in ("sdrgpu_fir_create", "sdrgpu_fir_process", "sdrgpu_fft_exec",
              "sdrgpu_stft_process", "sdrgpu_pll_process", "sdrgpu_firbank_process"):
        assert n in names


def test_library_exports_every_declared_symbol(sdr):
    L = sdr.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_binding_table_matches_header(sdr):
    from sdrgpu import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert bound == set(declared_functions())


def test_strerror_and_version(sdr):
    L = sdr.lib()
    assert L.sdrgpu_strerror(0) == b"no error"
    assert L.sdrgpu_strerror(6) == b"output buffer too small"
    assert L.sdrgpu_abi_version() == 1


def test_invalid_arguments_rejected_before_device(sdr):
    from sdrgpu import _lib
    L = sdr.lib()
    h = ctypes.c_void_p()
    taps = np.ones(4, np.float32)
    # null out-pointer / null taps / zero taps / zero decimation / f32 x c64 taps
    assert L.sdrgpu_fir_create(0, 1, 0, taps.ctypes.data, 4, 1, None) == _lib.ERR_INVALID
    assert L.sdrgpu_fir_create(0, 1, 0, None, 4, 1, ctypes.byref(h)) == _lib.ERR_INVALID
    assert L.sdrgpu_fir_create(0, 1, 0, taps.ctypes.data, 0, 1, ctypes.byref(h)) == _lib.ERR_INVALID
    assert L.sdrgpu_fir_create(0, 1, 0, taps.ctypes.data, 4, 0, ctypes.byref(h)) == _lib.ERR_INVALID
    assert L.sdrgpu_fir_create(0, 0, 1, taps.ctypes.data, 2, 1, ctypes.byref(h)) == _lib.ERR_INVALID
    assert L.sdrgpu_fir_process(None, None, 0, None, 0, None) == _lib.ERR_INVALID
    L.sdrgpu_fir_destroy(None)  # no-op like Drop on a null


def test_no_device_error_on_cpu_box(sdr):
    from sdrgpu import _lib
    if sdr.device_count() > 0:
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    taps = np.ones(4, np.float32)
    rc = sdr.lib().sdrgpu_fir_create(0, 1, 0, taps.ctypes.data, 4, 1, ctypes.byref(h))
    assert rc == _lib.ERR_NODEVICE and not h.value


def test_oracle_not_linked_into_product():
    so = os.path.join(ROOT, "unnamed-rust-sdr_amd", "libsdrgpu.so")
    data = open(so, "rb").read()
    assert b"oracle_" not in data and b"liboracle" not in data
