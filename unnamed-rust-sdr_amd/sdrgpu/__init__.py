"""sdrgpu -- MI355X-native FIR / FFT / PLL sample-stream core (host-side mirror).

Mirrors the reference crate's `filter`, `fft`, `resample` and `signal` API (agrif/unnamed-rust-sdr,
src/filter/mod.rs, src/fft.rs, src/signal/mod.rs) over the C ABI in include/sdrgpu.h.
All compute runs in libsdrgpu.so (hand-written HIP for gfx950); importing this package
without the built library raises ImportError.
"""
from . import _lib
from ._lib import C64, CU8, F32, SdrGpuError, device_count, lib
from . import device, fft, filter, resample, rtltcp, shard, signal  # noqa: F401

lib()  # fail loudly at import if the HIP library is missing

__all__ = ["device", "fft", "filter", "resample", "rtltcp", "shard", "signal", "C64", "CU8", "F32", "SdrGpuError", "device_count", "lib"]
