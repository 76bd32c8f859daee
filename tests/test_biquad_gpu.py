"""GPU parity: batched Biquad<C, f32> (sdrgpu_biquad_*) vs the oracle, bit-exact.

Reference: BiquadD::design (src/filter/biquad.rs:83-155), Biquad::new/apply (:25-56),
filter::Identity (src/filter/simple.rs:3-19), used as Signal::filter (src/signal/mod.rs:42-48)
-- e.g. the FM de-emphasis BiquadD::Lr (src/main.rs:52,75-81).  The kernel keeps the
reference's f32 operation order without contraction, so outputs must be array_equal.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RATE = 1.8e6
DESIGNS = [("LowPass", (80000.0, 0.7)), ("HighPass", (5000.0, 0.5)), ("BandPass", (19000.0, 5.0)),
           ("Notch", (60000.0, 2.0)), ("Lr", (75e-6,)), ("Identity", ())]


def make(sdr, name, args, sk, nch=1):
    f = sdr.filter
    d = f.Identity if name == "Identity" else getattr(f.BiquadD, name)(*args)
    return d, d.design(RATE, sample_kind=sk, nch=nch)


@pytest.mark.parametrize("sk", [0, 1], ids=["f32", "c64"])
@pytest.mark.parametrize("name,args", DESIGNS, ids=[d[0] for d in DESIGNS])
def test_biquad_bit_exact(sdr, oracle, name, args, sk):
    rng = np.random.default_rng(len(name) * 3 + sk)
    nch, n = 70, 5003
    d, bq = make(sdr, name, args, sk, nch)
    if sk:
        x = (rng.standard_normal((nch, n)) + 1j * rng.standard_normal((nch, n))).astype(np.complex64)
    else:
        x = rng.standard_normal((nch, n)).astype(np.float32)
    y = bq.process(x)
    c = d.to_c()
    if name != "Identity":
        np.testing.assert_array_equal(bq.coefs(), np.array(oracle.biquad_coefs(c.kind, c.freq, c.q, RATE),
                                                            np.float32))
    for ch in (0, 1, 63, 64, nch - 1):
        ref = x[ch] if name == "Identity" else oracle.biquad_run(c.kind, c.freq, c.q, RATE, x[ch])
        np.testing.assert_array_equal(y[ch], ref, err_msg=f"{name} ch {ch}")


def test_biquad_state_carry_reset_clone(sdr, oracle):
    rng = np.random.default_rng(4)
    d, bq = make(sdr, "LowPass", (80000.0, 0.7), 1, nch=3)
    x = (rng.standard_normal((3, 4000)) + 1j * rng.standard_normal((3, 4000))).astype(np.complex64)
    whole = bq.process(x)
    bq.reset()
    parts = [bq.process(x[:, a:b]) for a, b in ((0, 1), (1, 9), (9, 1000))]
    g = bq.clone()
    parts.append(bq.process(x[:, 1000:]))
    np.testing.assert_array_equal(np.concatenate(parts, axis=1), whole)
    np.testing.assert_array_equal(g.process(x[:, 1000:]), whole[:, 1000:])
    # Filter::apply on one sample of a 1-channel filter
    _, one = make(sdr, "Lr", (75e-6,), 0)
    v = one.apply(np.float32(1.0))
    c = sdr.filter.BiquadD.Lr(75e-6).to_c()
    assert v == oracle.biquad_run(c.kind, c.freq, c.q, RATE, np.array([1.0], np.float32))[0]


TP_CASES = [("LowPass", (20000.0, 0.7), 1.8e6), ("BandPass", (19000.0, 5.0), 1.8e6),
            ("Lr", (1.0 / 75e-6,), 144000.0), ("LowPass", (200.0, 0.7), 144000.0)]  # main.rs:52,57


def _signal(rng, sk, nch, n):
    if sk:
        return (rng.standard_normal((nch, n)) + 1j * rng.standard_normal((nch, n))).astype(np.complex64)
    return rng.standard_normal((nch, n)).astype(np.float32)


@pytest.mark.parametrize("sk", [0, 1], ids=["f32", "c64"])
@pytest.mark.parametrize("name,args,rate", TP_CASES, ids=["lp20k", "bp19k", "deemph", "lp200hz"])
def test_biquad_time_parallel_auto_bit_exact(sdr, oracle, name, args, rate, sk):
    """A few long streams (the de-emphasis / pilot-filter shape of src/main.rs:52-60, and the
    PLL's lock filter at 1.8 Msps) through the automatic time-parallel plan: segments run at
    once after a warm-up sized from the design's slower pole, verified bit for bit and
    recomputed where they miss -- outputs array_equal to the oracle's serial Biquad::apply,
    over two calls (state carried), and to the handle's own serial pass."""
    rng = np.random.default_rng(90 + sk + int(rate) % 7)
    nch, n, cut = 3, 1200000, 800000
    d = getattr(sdr.filter.BiquadD, name)(*args)
    bq = d.design(rate, sample_kind=sk, nch=nch)
    seg, warm = bq.time_parallel_plan(cut)
    assert seg > 0 and warm >= 64 and seg >= 4 * warm, (seg, warm)
    x = _signal(rng, sk, nch, n)
    y1 = bq.process(x[:, :cut])
    segs, rec = bq.last_time_parallel()
    assert segs >= 2 and 0 <= rec <= nch * (segs - 1)
    y = np.concatenate([y1, bq.process(x[:, cut:])], axis=1)
    c = d.to_c()
    for ch in range(nch):
        np.testing.assert_array_equal(y[ch], oracle.biquad_run(c.kind, c.freq, c.q, rate, x[ch]),
                                      err_msg=f"{name} ch {ch}")
    serial = d.design(rate, sample_kind=sk, nch=nch)
    serial.set_time_parallel(-1)
    assert serial.time_parallel_plan(n)[0] == 0
    np.testing.assert_array_equal(serial.process(x), y)


@pytest.mark.parametrize("seg,warm", [(4096, 8), (1000, 200), (8192, 100000), (2048, 1024)],
                         ids=["mostly-recomputed", "ragged", "warm-reaches-start", "converging"])
def test_biquad_time_parallel_forced(sdr, oracle, seg, warm):
    """Forced segment / warm-up lengths on 70 complex channels: a warm-up so short that nearly
    every segment misses its guess (the re-run and serial repair paths), a segment length that
    leaves a ragged last segment, a warm-up reaching back to the block start (exact guesses)
    and a converging one; array_equal to the oracle, state carried into a second block."""
    rng = np.random.default_rng(seg + warm)
    nch, n = 70, 30011
    d = sdr.filter.BiquadD.LowPass(20000.0, 0.7)
    bq = d.design(RATE, sample_kind=1, nch=nch)
    bq.set_time_parallel(seg, warm)
    assert bq.time_parallel_plan(20000) == ((seg + 7) // 8 * 8, warm)
    x = _signal(rng, 1, nch, n)
    y1 = bq.process(x[:, :20000])
    segs, rec = bq.last_time_parallel()
    assert segs == -(-20000 // ((seg + 7) // 8 * 8))
    if warm >= 20000:
        assert rec == 0
    if warm == 8:
        assert rec > nch
    y = np.concatenate([y1, bq.process(x[:, 20000:])], axis=1)
    c = d.to_c()
    for ch in (0, 1, 33, 64, nch - 1):
        np.testing.assert_array_equal(y[ch], oracle.biquad_run(c.kind, c.freq, c.q, RATE, x[ch]),
                                      err_msg=f"ch {ch}")


def test_biquad_time_parallel_not_for_identity_integrator_or_many_channels(sdr):
    """Identity has no recurrence, Lr(75e-6) at 144 kHz rounds its pole to exactly 1.0 in f32
    (an integrator: two trajectories never meet), the pilot's LowPass(20 Hz) at 144 kHz has its
    poles within 0.07 % of the unit circle, and 65536 channels already fill the device: serial
    plans (an explicit set_time_parallel still applies)."""
    f = sdr.filter
    ident = f.Identity.design(RATE, sample_kind=0, nch=1)
    assert ident.time_parallel_plan(1 << 20)[0] == 0
    integ = f.BiquadD.Lr(75e-6).design(144000.0, sample_kind=0, nch=1)
    assert integ.coefs()[3] == 1.0 and integ.time_parallel_plan(1 << 20)[0] == 0
    pilot = f.BiquadD.LowPass(20.0, 0.7).design(144000.0, sample_kind=0, nch=1)
    assert pilot.time_parallel_plan(1 << 24) == (0, 0)
    pilot.set_time_parallel(1 << 20, 1 << 16)
    assert pilot.time_parallel_plan(1 << 24) == (1 << 20, 1 << 16)
    many = f.BiquadD.LowPass(20000.0, 0.7).design(RATE, sample_kind=0, nch=65536)
    assert many.time_parallel_plan(1 << 16)[0] == 0


def test_biquad_time_parallel_strided_device_rows(sdr, oracle):
    """Time-parallel blocks on device rows with leading dimensions larger than the block (ld_in
    = n + 37, ld_out = n + 5, as a caller's channel-major buffers give them), c64 and f32,
    two blocks with the state carried: array_equal to the oracle."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(77)
    d = sdr.filter.BiquadD.LowPass(20000.0, 0.7)
    for sk, dt in ((1, np.complex64), (0, np.float32)):
        nch, n = 2, 300000
        bq = d.design(RATE, sample_kind=sk, nch=nch)
        assert bq.time_parallel_plan(n // 2)[0] > 0
        x = _signal(rng, sk, nch, n)
        ldi, ldo = n // 2 + 37, n // 2 + 5
        halves = []
        for h in range(2):
            xi = np.zeros((nch, ldi), dt)
            xi[:, :n // 2] = x[:, h * (n // 2):(h + 1) * (n // 2)]
            dx = DeviceBuffer.from_numpy(xi)
            dy = DeviceBuffer.empty(nch * ldo, dt)
            bq.process_dev(dx.ptr, ldi, n // 2, dy.ptr, ldo)
            bq.sync()
            assert bq.last_time_parallel()[0] >= 2
            halves.append(dy.download(nch * ldo, dt).reshape(nch, ldo)[:, :n // 2])
        y = np.concatenate(halves, axis=1)
        c = d.to_c()
        for ch in range(nch):
            np.testing.assert_array_equal(y[ch], oracle.biquad_run(c.kind, c.freq, c.q, RATE, x[ch]))


def test_biquad_in_place_long_block(sdr, oracle):
    """An in-place process_dev call (d_out == d_in) on a block long enough for the time-parallel
    plan: the handle runs its serial pass (the segment kernels re-read inputs after outputs are
    stored), so the result is still Biquad::apply's (biquad.rs:42-56), f32 and c64, state
    carried into a second in-place block."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(78)
    d = sdr.filter.BiquadD.LowPass(20000.0, 0.7)
    for sk, dt in ((1, np.complex64), (0, np.float32)):
        nch, n = 2, 400000
        bq = d.design(RATE, sample_kind=sk, nch=nch)
        assert bq.time_parallel_plan(n // 2)[0] > 0
        x = _signal(rng, sk, nch, n)
        halves = []
        for h in range(2):
            dx = DeviceBuffer.from_numpy(np.ascontiguousarray(x[:, h * (n // 2):(h + 1) * (n // 2)]))
            bq.process_dev(dx.ptr, n // 2, n // 2, dx.ptr, n // 2)
            bq.sync()
            assert bq.last_time_parallel()[0] == 0  # serial pass
            halves.append(dx.download(nch * (n // 2), dt).reshape(nch, n // 2))
        y = np.concatenate(halves, axis=1)
        c = d.to_c()
        for ch in range(nch):
            np.testing.assert_array_equal(y[ch], oracle.biquad_run(c.kind, c.freq, c.q, RATE, x[ch]))
