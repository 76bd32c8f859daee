"""Host-side mirror of the reference `Signal` trait (src/signal/mod.rs:13-123) over sdrgpu.

The reference pulls one sample at a time through adapter structs; here a Signal yields
BLOCKS (numpy arrays) and every GPU-backed stage carries its stream state across blocks,
so results equal the sample-by-sample reference for any block size.  Combinators keep the
reference names and argument meaning:

  filter(design)     adapters::Filter (adapters/mod.rs:66-100): FIR taps / filter.Fir
                     (fir.rs:36-58) or filter.PllDesign (pll.rs:39-61, output Option<f32>
                     as (value-or-0.0, locked) blocks like src/main.rs:49 unwraps it)
  decimate(rate)     Decimate (adapters/mod.rs:13-41): wait = round(rate_in / rate), keeps
                     upstream indices wait-1, 2wait-1, ...; rate() stays the UPSTREAM rate
                     (the reference quirk, :38-40).  A decimate directly after a FIR filter
                     is fused into the FIR kernel (only kept outputs are computed).
  window(duration)   Window (adapters/mod.rs:270-303), cap = round(duration * rate)
  .decimate(..).map(fft)  the live.rs STFT pattern -> one GPU Stft stage
  resample(rate), resample_with(typ, rate)
                     adapters::Resample (adapters/resample.rs:17-82): 4096-frame buffers
                     through resample.SampleRate (GPU sinc / ZOH / linear); rate() = the new rate
  map(f), take(duration), skip(duration), iter(), collect()

Sources: from_array (FromIter, sources.rs:6-36), freq (sources.rs:196-221), freq_sweep
(sources.rs:116-194), impulse (sources.rs:223-257).
"""
from __future__ import annotations

import math
from typing import Callable, Iterator, Optional

import numpy as np

from . import _lib
from . import filter as _filter
from . import fft as _fft
from . import resample as _resample

DEFAULT_BLOCK = 1 << 16


# rtl_tcp blocks (sample_kind CU8) are raw interleaved I/Q bytes, 2 per sample: the sample-
# counting adapters below index them in sample units (byte pairs), never single bytes
def _nsamples(b, kind) -> int:
    return b.size // 2 if kind == _lib.CU8 else len(b)


def _pairs(b, kind):
    return np.asarray(b).reshape(-1, 2) if kind == _lib.CU8 else b


def _unpairs(b, kind):
    return b.reshape(-1) if kind == _lib.CU8 else b


def _cu8_values(b) -> np.ndarray:
    """RtlTcpSignal::next (src/rtltcp.rs:156-164): (v - 128) / 128, for host-side adapters
    that hand samples to arbitrary Python code (the GPU stages read the bytes directly)."""
    v = (np.asarray(b, np.float32).reshape(-1, 2) - np.float32(128.0)) / np.float32(128.0)
    return (v[:, 0] + 1j * v[:, 1]).astype(np.complex64)


class Signal:
    def __init__(self, rate: float, blocks: Callable[[], Iterator[np.ndarray]],
                 sample_kind: Optional[int] = None, _fir: Optional[dict] = None):
        self._rate = float(rate)
        self._blocks = blocks
        self.sample_kind = sample_kind
        self._fir = _fir  # pending FIR stage that a following decimate may fuse into

    # ---- Signal::rate / iteration ----
    def rate(self) -> float:
        return self._rate

    def blocks(self) -> Iterator[np.ndarray]:
        return self._blocks()

    def iter(self):
        """Signal::iter: samples one by one (rtl_tcp bytes as Complex<f32>, rtltcp.rs:156-164)."""
        for b in self.blocks():
            yield from (_cu8_values(b) if self.sample_kind == _lib.CU8 else b)

    def collect(self) -> np.ndarray:
        bl = [(_cu8_values(b) if self.sample_kind == _lib.CU8 else b) for b in self.blocks()]
        return np.concatenate(bl) if bl else np.zeros(0)

    # ---- combinators ----
    def filter(self, design, block_kind=None) -> "Signal":
        if isinstance(design, _filter.PllDesign):
            return self._pll(design)
        if isinstance(design, (list, tuple, np.ndarray)):
            design = _filter.Fir(np.asarray(design))
        if isinstance(design, _filter.Fir):
            return self._fir_stage(design, 1)
        raise _lib.SdrGpuError(_lib.ERR_UNSUPPORTED,
                               f"Signal.filter: {type(design).__name__} is not on the GPU path")

    def _fir_stage(self, fir: "_filter.Fir", decim: int) -> "Signal":
        up = self
        sk = self.sample_kind if self.sample_kind is not None else (
            _lib.C64 if fir.tap_kind == _lib.C64 else _lib.F32)

        def gen():
            f = fir.with_decim(decim).design(up.rate(), sample_kind=sk)
            for b in up.blocks():
                y = f.process(b)
                if y.size:
                    yield y
        # rtl_tcp bytes in, Complex<f32> out: downstream stages see C64 samples
        out_kind = _lib.C64 if sk == _lib.CU8 else sk
        return Signal(self._rate, gen, out_kind, _fir={"up": up, "fir": fir, "decim": decim})

    def _pll(self, design: "_filter.PllDesign") -> "Signal":
        up = self

        def gen():
            p = design.design(up.rate())
            for b in up.blocks():
                if up.sample_kind == _lib.CU8:  # rtl_tcp bytes straight into the PLL
                    out, locked = p.process_u8(b)
                else:
                    out, locked = p.process(np.asarray(b, np.complex64))
                yield np.rec.fromarrays([out, locked.astype(bool)], names="value,locked")
        return Signal(self._rate, gen, None)

    def decimate(self, rate: float) -> "Signal":
        wait = int(round(self._rate / rate))
        if wait < 1:
            raise _lib.SdrGpuError(_lib.ERR_INVALID, "decimate: rate above the input rate")
        if self._fir is not None and self._fir["decim"] == 1:
            # Filter(..).decimate(..): fuse -> only kept outputs are computed on the GPU
            return self._fir["up"]._fir_stage(self._fir["fir"], wait)
        if getattr(self, "_window", None) is not None:
            return _WindowDecimate(self, self._window, wait)
        up = self
        sk = self.sample_kind

        def gen():
            phase = 0  # samples consumed mod wait
            for b in up.blocks():
                first = (wait - 1 - phase) % wait
                yield _unpairs(_pairs(b, sk)[first::wait], sk)
                phase = (phase + _nsamples(b, sk)) % wait
        return Signal(self._rate, gen, sk)  # Decimate::rate quirk (:38-40)

    def resample(self, rate: float) -> "Signal":
        """Signal::resample (src/signal/mod.rs:78-84): SincBestQuality (this library's own
        sinc table)."""
        return self.resample_with(_resample.ConverterType.SincBestQuality, rate)

    def resample_with(self, typ, rate: float) -> "Signal":
        """Signal::resample_with -> adapters::Resample (adapters/resample.rs:17-82): refill a
        4096-frame buffer from upstream, SampleRate::process(ratio, buffer, capacity 4096),
        drop the used frames, stop when a call has neither input nor output."""
        up = self
        buffer_size = 4096
        # ratio: rate as f64 / signal.rate() as f64, both f32 in the reference
        ratio = float(np.float32(rate)) / float(np.float32(up.rate()))

        def gen():
            sr = None
            buf = None
            cplx = False
            it = iter(up.blocks())
            pending = []  # upstream frames not yet in the buffer
            exhausted = False
            while True:
                while not exhausted and (buf is None or buf.shape[0] < buffer_size):
                    if pending:
                        need = buffer_size - (0 if buf is None else buf.shape[0])
                        take, rest = pending[0][:need], pending[0][need:]
                        buf = take if buf is None else np.concatenate([buf, take])
                        pending = [rest] if rest.shape[0] else []
                        continue
                    b = next(it, None)
                    if b is None:
                        exhausted = True
                        break
                    # rtl_tcp bytes reach SampleRate as the Complex<f32> samples
                    # RtlTcpSignal::next yields (rtltcp.rs:156-164), two channels
                    b = _cu8_values(b) if up.sample_kind == _lib.CU8 else np.asarray(b)
                    if sr is None:
                        cplx = np.iscomplexobj(b)
                        ch = 2 if cplx else (1 if b.ndim == 1 else b.shape[1])
                        sr = _resample.SampleRate(typ, ch)
                    pending.append(_resample._frames(b, sr.channels()))
                if sr is None:
                    return
                if buf is None:
                    buf = np.zeros((0, sr.channels()), np.float32)
                used, out = sr.process(ratio, buf, buffer_size)
                if buf.shape[0] == 0 and out.shape[0] == 0:
                    return
                buf = buf[used:]
                if out.shape[0]:
                    if cplx:
                        yield out.view(np.complex64).reshape(-1)
                    elif out.shape[1] == 1:
                        yield out.reshape(-1)
                    else:
                        yield out
        # the output is converted samples: Complex<f32> for complex (or rtl_tcp) input, f32 for
        # mono, frames of `channels` f32 otherwise -- never raw CU8 byte pairs
        if self.sample_kind in (_lib.C64, _lib.CU8):
            out_kind = _lib.C64
        elif self.sample_kind == _lib.F32:
            out_kind = _lib.F32
        else:
            out_kind = None
        return Signal(float(np.float32(rate)), gen, out_kind)

    def window(self, duration: float) -> "Signal":
        cap = int(round(duration * self._rate))
        s = Signal(self._rate, self._blocks, self.sample_kind)
        s._window = cap
        return s

    def map(self, fn: Callable) -> "Signal":
        """Signal::map: fn sees Complex<f32> samples for rtl_tcp input (rtltcp.rs:156-164)."""
        up = self

        def gen():
            for b in up.blocks():
                yield fn(_cu8_values(b) if up.sample_kind == _lib.CU8 else b)
        return Signal(self._rate, gen, None)

    def take(self, duration: float) -> "Signal":
        n = int(round(self._rate * duration))
        up = self
        sk = self.sample_kind

        def gen():
            left = n
            for b in up.blocks():
                if left <= 0:
                    return
                yield _unpairs(_pairs(b, sk)[:left], sk)
                left -= _nsamples(b, sk)
        return Signal(self._rate, gen, sk)

    def skip(self, duration: float) -> "Signal":
        n = int(round(self._rate * duration))
        up = self
        sk = self.sample_kind

        def gen():
            left = n
            for b in up.blocks():
                nb = _nsamples(b, sk)
                if left >= nb:
                    left -= nb
                    continue
                yield _unpairs(_pairs(b, sk)[left:], sk)
                left = 0
        return Signal(self._rate, gen, sk)


class _WindowDecimate(Signal):
    """window(N).decimate(rate): frames x[(j+1)hop - N .. (j+1)hop) (adapters/mod.rs:277-299).
    .map(fft) on it runs the GPU STFT; other maps get the raw frames."""

    def __init__(self, up: Signal, cap: int, hop: int):
        self.up, self.cap, self.hop = up, cap, hop

        def frames():
            buf = np.zeros(cap, np.complex64)
            phase = 0
            for b in up.blocks():
                if up.sample_kind == _lib.CU8:
                    b = _cu8_values(b)
                for v in b:
                    buf = np.roll(buf, -1)
                    buf[-1] = v
                    phase += 1
                    if phase == hop:
                        phase = 0
                        yield buf.copy()[None, :]
        super().__init__(up.rate(), frames, None)

    def map(self, fn: Callable) -> Signal:
        if fn is fft or fn is _fft.fft:
            up, cap, hop = self.up, self.cap, self.hop

            def gen():
                # rtl_tcp bytes go to the GPU as they are (converted in the frame load)
                kind = _lib.CU8 if up.sample_kind == _lib.CU8 else _lib.C64
                s = _fft.Stft(cap, hop, input_kind=kind)
                for b in up.blocks():
                    y = s.process(b)
                    if y.shape[0]:
                        yield y
            return Signal(self._rate, gen, None)
        return super().map(fn)


def fft(frames):
    """Marker for .map(fft) on window+decimate (the examples/live.rs STFT)."""
    return np.stack([_fft.fft(f, 1.0)[1] for f in np.atleast_2d(frames)])


# ---------------------------------------------------------------- sources
_LIBM = None


def _polar_unit(ph: np.ndarray) -> np.ndarray:
    """Complex::from_polar(&1.0, &ph) with glibc cosf / sinf -- what Rust's f32::cos / sin
    call on Linux (numpy's float32 cos / sin differ from glibc by an ulp now and then)."""
    import ctypes
    global _LIBM
    if _LIBM is None:
        _LIBM = ctypes.CDLL("libm.so.6")
        for fn in (_LIBM.cosf, _LIBM.sinf):
            fn.restype = ctypes.c_float
            fn.argtypes = [ctypes.c_float]
    out = np.empty(ph.size, np.complex64)
    for i, p in enumerate(ph.tolist()):
        out[i] = complex(_LIBM.cosf(p), _LIBM.sinf(p))
    return out

def from_array(rate: float, x, block: int = DEFAULT_BLOCK,
               sample_kind: Optional[int] = None) -> Signal:
    """signal::from_iter (sources.rs:6-36) over an array, `block` samples per block.
    sample_kind=CU8 marks x as raw rtl_tcp I/Q bytes (2 per sample), as RtlTcp.listen()
    yields them."""
    x = np.asarray(x)
    sk = sample_kind if sample_kind is not None else (
        _lib.C64 if np.iscomplexobj(x) else _lib.F32)
    if sk == _lib.CU8:
        x = np.ascontiguousarray(x, np.uint8).reshape(-1)
        step = 2 * block
    else:
        step = block

    def gen():
        for i in range(0, len(x), step):
            yield x[i:i + step]
    return Signal(rate, gen, sk)


def freq(rate: float, f: float, phase: float, n: int, block: int = DEFAULT_BLOCK) -> Signal:
    """signal::freq (sources.rs:196-221) for n samples (FreqSweep::next arithmetic in f32)."""
    two_pi = np.float32(2.0) * np.float32(np.pi)
    dt = np.float32(1.0) / np.float32(rate)
    ff = np.float32(f)
    nph = np.float32(phase) / two_pi
    phs = np.empty(n, np.float32)
    for i in range(n):
        nph = np.float32(nph + np.float32(dt * ff))
        nph = np.float32(nph - np.trunc(nph))
        phs[i] = np.float32(two_pi * nph)
    return from_array(rate, _polar_unit(phs), block)


USIZE_MAX = (1 << 64) - 1


def _as_usize(v) -> int:
    """`v.round() as usize` for an f32 v (FreqSweep::new, sources.rs:133-134): round half away
    from zero, then the saturating cast (negative -> 0).  |v| + 0.5 is formed in f64 -- in
    f32 it would itself round (2^23 + 1 -> 2^23 + 2, 0.49999997 -> 1).  Rust's float -> int
    `as` saturates: NaN and negatives give 0 (e.g. freq_sweep with df = 0 and rate = 0, where
    inf * 0 = NaN: an empty sweep), +inf gives usize::MAX."""
    v = float(np.float32(v))
    if not v > 0:           # NaN, -0, 0 and negatives
        return 0
    if math.isinf(v):
        return USIZE_MAX
    return min(int(math.floor(v + 0.5)), USIZE_MAX)


def freq_sweep(rate: float, df: float, warmup: bool, start: float, end: float,
               block: int = DEFAULT_BLOCK) -> Signal:
    """signal::freq_sweep(rate, df, warmup, start..end) (sources.rs:181-194) through
    FreqSweep::new / next (:129-174) in f32: blocks are records (freq, value) like the
    reference's (f32, Complex<f32>) samples; the sweep ends after its length."""
    f32 = np.float32
    two_pi = f32(2.0) * f32(np.pi)
    dfdt = f32(df) * f32(df)
    if start > end:
        dfdt = -dfdt
    endt = (f32(end) - f32(start)) / dfdt
    warmupt = f32(1.0) / f32(df) if warmup else f32(0.0)
    fend_t = f32(warmupt + endt)

    as_usize = _as_usize
    rate32 = f32(rate)
    fstart = as_usize(f32(warmupt * rate32))
    fend = as_usize(f32(fend_t * rate32))
    n = fend
    if n == USIZE_MAX:  # an unbounded sweep (Rust's lazy iterator would never end)
        raise _lib.SdrGpuError(_lib.ERR_INVALID, "freq_sweep: unbounded length (+inf samples)")
    dt = f32(1.0) / rate32
    fr = f32(start)
    nph = f32(0.0) / two_pi
    freqs = np.empty(n, np.float32)
    phs = np.empty(n, np.float32)
    for i in range(n):
        d = dfdt
        if fstart > 0:
            fstart -= 1
            d = f32(0.0)
        if fend > 0:
            fend -= 1
        else:
            d = f32(0.0)
        fr = f32(fr + f32(dt * d))
        nph = f32(nph + f32(dt * fr))
        nph = f32(nph - np.trunc(nph))
        phs[i] = f32(two_pi * nph)
        freqs[i] = fr
    rec = np.rec.fromarrays([freqs, _polar_unit(phs)], names="freq,value")

    def gen():
        for i in range(0, n, block):
            yield rec[i:i + block]
    return Signal(rate, gen, None)


def impulse(rate: float, n: int, complex_: bool = False, block: int = DEFAULT_BLOCK) -> Signal:
    """signal::impulse (sources.rs:223-257): 1 then zeros (n samples)."""
    x = np.zeros(n, np.complex64 if complex_ else np.float32)
    if n:
        x[0] = 1
    return from_array(rate, x, block)
