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
