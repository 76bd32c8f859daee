"""The reference binary's whole FM stereo chain (src/main.rs:33-81) through sdrgpu.fm.receiver
-- GPU PLL on the rtl_tcp bytes, SincFastest resampler, pilot-PLL stereo difference,
SincBestQuality resampler, de-emphasis bank -- against the same chain composed from the oracle's
restatements, bit for bit.

The input is a synthetic FM stereo broadcast: (L + R) + 0.1 pilot(19 kHz) + (L - R) at 38 kHz
DSB, frequency-modulated with 75 kHz deviation at 1.8 Msps and quantised to rtl_tcp's u8 I/Q.
The oracle side calls each SampleRate once over the whole stream (plus the end-of-input flush);
the GPU side runs the Signal adapter's 4096-frame buffer refills (src/signal/adapters/
resample.rs:17-82) -- the sinc converters are partition-invariant, so the two must agree.
The resampler tables are this library's own (parity unpinned against libsamplerate)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RATE = 1.8e6


def fm_stereo_u8(n, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / RATE
    left = 0.4 * np.sin(2 * np.pi * 440.0 * t)
    right = 0.4 * np.sin(2 * np.pi * 1250.0 * t + 0.3)
    pilot = np.cos(2 * np.pi * 19000.0 * t)
    comp = 0.45 * (left + right) + 0.1 * pilot + 0.45 * (left - right) * np.cos(2 * np.pi * 38000.0 * t)
    phase = 2 * np.pi * 75000.0 * np.cumsum(comp) / RATE
    iq = np.exp(1j * phase) * 0.8 + 0.02 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    raw = np.empty(2 * n, np.uint8)
    raw[0::2] = np.clip(np.round(iq.real * 127.5 + 127.5), 0, 255).astype(np.uint8)
    raw[1::2] = np.clip(np.round(iq.imag * 127.5 + 127.5), 0, 255).astype(np.uint8)
    return raw


def _src_all(oracle, conv, ch, ratio, x):
    """SampleRate::process over the whole input, then empty calls until the sinc flush ends."""
    sr = oracle.SampleRate(conv, ch)
    out = []
    used, y = sr.process(ratio, x, x.shape[0] * 4 + 64)
    assert used == x.shape[0]
    out.append(y)
    while True:
        _, y = sr.process(ratio, x[:0], 4096)
        if y.shape[0] == 0:
            break
        out.append(y)
    return np.concatenate(out)


def oracle_chain(oracle, raw, fm_mod):
    dev = np.float32(75000.0)
    # main.rs:41-49: PLL on the converted bytes, None -> 0.0, / 75000
    p = oracle.pll_params(0.0, 0.035, RATE, (1, 80000.0, 0.7), (0, 0.0, 0.0), (1, 20000.0, 0.7))
    out, locked = oracle.pll_batch(p, oracle.u8_to_c64(raw)[None, :])
    v = np.where(locked[0] != 0, out[0], np.float32(0.0)).astype(np.float32) / dev
    # main.rs:50: SincFastest to 144 kHz (ratio as adapters/resample.rs computes it)
    r1 = float(np.float32(144000.0)) / float(np.float32(RATE))
    a = _src_all(oracle, 2, 1, r1, v[:, None])[:, 0]
    # main.rs:54-69: pilot PLL at 144 kHz, (mono, diff)
    pp = oracle.pll_params(19000.0, 0.0002, 144000.0, (1, 200.0, 0.7), (1, 20.0, 0.7), (1, 20.0, 0.7))
    mono, diff, _ = oracle.pll_stereo(pp, a)
    # main.rs:71: SincBestQuality to 48 kHz, two channels
    r2 = float(np.float32(48000.0)) / float(np.float32(144000.0))
    b = _src_all(oracle, 0, 2, r2, np.stack([mono, diff], axis=1))
    # main.rs:52,73-81: de-emphasis on each, (mono + diff, mono - diff)
    c = fm_mod.deemphasis().to_c()
    md = oracle.biquad_run(c.kind, c.freq, c.q, 48000.0, np.ascontiguousarray(b[:, 0]))
    dd = oracle.biquad_run(c.kind, c.freq, c.q, 48000.0, np.ascontiguousarray(b[:, 1]))
    return np.stack([md + dd, md - dd], axis=1), locked[0]


@pytest.mark.parametrize("block", [4096, 100003])
def test_main_rs_fm_stereo_chain_bit_exact(sdr, oracle, block):
    from sdrgpu import _lib, fm
    from sdrgpu.signal import from_array
    n = 540000  # 0.3 s of air
    raw = fm_stereo_u8(n)
    rtl = from_array(RATE, raw, block=block, sample_kind=_lib.CU8)
    got = np.concatenate(list(fm.receiver(rtl).blocks()), axis=0)
    ref, locked = oracle_chain(oracle, raw, fm)
    assert locked.mean() > 0.9, "the discriminator PLL should lock on this signal"
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.array_equal(got, ref)
    # the audio is there: the mono sum carries the 440 Hz and 1250 Hz tones
    tail = got[got.shape[0] // 2:]
    spec = np.abs(np.fft.rfft(tail[:, 0] + tail[:, 1]))
    f = np.fft.rfftfreq(tail.shape[0], 1 / 48000.0)
    top = f[np.argsort(spec[5:])[-2:] + 5]
    assert all(min(abs(t - 440.0), abs(t - 1250.0)) < 30.0 for t in top), top
