"""The reference binary's FM stereo receiver chain (src/main.rs:33-81) on the GPU stages.

`receiver(rtl)` takes what `rtl.listen()` yields -- an rtl_tcp u8 I/Q Signal at 1.8 Msps
(sample_kind CU8, e.g. `sdrgpu.rtltcp.RtlTcp(...).listen()` or `signal.from_array(...,
sample_kind=CU8)`) -- and returns the 48 kHz (left, right) Signal main.rs writes to the WAV
file or the audio card, stage for stage:

  main.rs:41-47   PLL FM discriminator on the raw bytes  -> Pll (CU8 input), None -> 0.0, / 75000
  main.rs:48      resample_with(SincFastest, 144 kHz)    -> SampleRate (this library's sinc table)
  main.rs:54-69   19 kHz pilot PLL, (mono, diff)         -> Pll stereo-difference output mode
  main.rs:71      resample(48 kHz)                       -> SampleRate SincBestQuality, 2 channels
  main.rs:52,73-81 de-emphasis Lr on mono and diff       -> one 2-channel Biquad bank
                   -> (mono + diff, mono - diff)

The `block(0.1)` stages are the reference's threading (src/signal/adapters/block.rs) and
`monitor` prints; neither changes a sample, so they are not stages here.  Every GPU stage is
bit-exact to its oracle restatement (tests/test_fm_chain_gpu.py checks the whole chain); the
two resamplers use this library's sinc tables, so that part is parity-unpinned against the
real libsamplerate."""
import numpy as np

from . import _lib
from . import filter as _filter
from . import resample as _resample

RATE = 1800000.0
DEVIATION = 75000.0


def discriminator_design() -> "_filter.PllDesign":
    """main.rs:41-46."""
    f = _filter
    return f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                       f.BiquadD.LowPass(20000.0, 0.7))


def pilot_design() -> "_filter.PllDesign":
    """main.rs:54-60."""
    f = _filter
    return f.PllDesign(19000.0, 0.0002, f.BiquadD.LowPass(200.0, 0.7), f.BiquadD.LowPass(20.0, 0.7),
                       f.BiquadD.LowPass(20.0, 0.7))


def deemphasis() -> "_filter.BiquadD":
    """main.rs:52: BiquadD::Lr(1.0 / (75.0 * 0.001 * 0.001)) -- f32 arithmetic."""
    return _filter.BiquadD.Lr(float(np.float32(1.0) / (np.float32(75.0) * np.float32(0.001) * np.float32(0.001))))


def receiver(rtl):
    """src/main.rs:48-81 over `rtl` (rtl_tcp bytes at 1.8 Msps): Signal of (n, 2) f32 frames
    (left, right) at 48 kHz.  Like every other stage, the pilot PLL and the de-emphasis bank
    are built inside the generators, so each iteration of the returned Signal starts from
    fresh filter state (the reference builds its chain once per run, main.rs:33-81)."""
    from .signal import Signal
    if rtl.sample_kind != _lib.CU8:
        raise _lib.SdrGpuError(_lib.ERR_INVALID, "fm.receiver: expects rtl_tcp u8 I/Q (CU8)")
    dev = np.float32(DEVIATION)
    fm = rtl.filter(discriminator_design()).map(
        lambda r: np.where(r["locked"], r["value"], np.float32(0.0)).astype(np.float32) / dev)
    audio = fm.resample_with(_resample.ConverterType.SincFastest, 48000.0 * 3.0)

    def stereo():  # main.rs:54-69 with the pilot PLL on the GPU (state carried per block)
        pilot = pilot_design().design(audio.rate())
        for v in audio.blocks():
            mono, diff, _ = pilot.stereo(np.asarray(v, np.float32))
            yield np.stack([mono, diff], axis=1)

    md = Signal(audio.rate(), stereo, None).resample(48000.0)

    def out():  # main.rs:75-81
        bank = deemphasis().design(md.rate(), sample_kind=_lib.F32, nch=2)
        for frames in md.blocks():
            y = bank.process(np.ascontiguousarray(np.asarray(frames, np.float32).T))
            yield np.stack([y[0] + y[1], y[0] - y[1]], axis=1)

    return Signal(md.rate(), out, None)
