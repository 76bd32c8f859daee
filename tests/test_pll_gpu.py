"""GPU parity: batched PLL FM demod (Pll::apply, src/filter/pll.rs:70-85) vs the oracle.

The loop is a chaotic nonlinear recurrence on noisy input (a 1-ulp change in one sample
moves the next cycle slip), so the GPU kernel restates the reference arithmetic exactly
(no contraction, reference operation order, glibc-identical sinf/cosf/atan2f -- see
csrc/libm_glibc.h and tests/test_libm_restatement.py).  Parity is therefore BIT-EXACT:
outputs (None -> 0.0, src/main.rs:49) and lock masks equal the oracle's."""
import numpy as np
import pytest

from conftest import assert_parity

pytestmark = pytest.mark.gpu

RATE = 1.8e6


def fm_channels(rng, nch, n, dev=40e3, fmod=1e3, noise=0.05):
    """Per-channel FM: carrier in +-100 kHz, +-40 kHz deviation at 1 kHz."""
    t = np.arange(n) / RATE
    out = np.empty((nch, n), np.complex64)
    for c in range(nch):
        fc = rng.uniform(-100e3, 100e3)
        ph = 2 * np.pi * (fc * t + dev / fmod * np.sin(2 * np.pi * fmod * t + rng.uniform(0, 6)))
        out[c] = (np.exp(1j * ph) + noise * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
                  ).astype(np.complex64)
    return out


def main_rs_design(sdr):
    f = sdr.filter
    # src/main.rs:41-46
    return f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.Identity,
                       f.BiquadD.LowPass(20000.0, 0.7))


def oracle_params(oracle, ref=0.0, gain=0.035, loopf=(1, 80000.0, 0.7), outf=(0, 0.0, 0.0),
                  lockf=(1, 20000.0, 0.7)):
    return oracle.pll_params(ref, gain, RATE, loopf, outf, lockf)


def check(out, lk, ref_out, ref_lk, what):
    assert np.array_equal(lk, ref_lk), f"{what}: lock mask differs in {np.sum(lk != ref_lk)} samples"
    if not np.array_equal(out, ref_out):
        bad = np.argwhere(out != ref_out)
        raise AssertionError(f"{what}: {len(bad)} outputs differ, first at {bad[0]}")
    assert_parity(out, ref_out, what=what)


def test_pll_fm_batch_parity(sdr, oracle):
    rng = np.random.default_rng(1)
    nch, n = 64, 40000
    x = fm_channels(rng, nch, n)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    out, lk = pll.process(x)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), x, nthreads=8)
    check(out, lk, ref_out, ref_lk, "main.rs PLL")


def test_pll_examples_design_with_output_filter(sdr, oracle):
    # examples/pll.rs:9-15: output filter LowPass(20 kHz) instead of Identity
    f = sdr.filter
    rng = np.random.default_rng(2)
    nch, n = 16, 30000
    x = fm_channels(rng, nch, n)
    d = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.BiquadD.LowPass(20000.0, 0.7),
                    f.BiquadD.LowPass(20000.0, 0.7))
    out, lk = d.design(RATE, nch=nch).process(x)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle, outf=(1, 20000.0, 0.7)), x)
    check(out, lk, ref_out, ref_lk, "examples/pll.rs PLL")


def test_pll_reference_and_lr_filters(sdr, oracle):
    # pilot-style PLL (src/main.rs:55-60): nonzero reference, different gains / filters
    f = sdr.filter
    rng = np.random.default_rng(3)
    nch, n = 8, 20000
    t = np.arange(n) / RATE
    x = np.stack([np.exp(2j * np.pi * (19000.0 + 50 * c) * t) for c in range(nch)]).astype(np.complex64)
    d = f.PllDesign(19000.0, 0.0002, f.BiquadD.LowPass(200.0, 0.7), f.BiquadD.Lr(1000.0),
                    f.BiquadD.HighPass(20.0, 0.7))
    out, lk = d.design(RATE, nch=nch).process(x)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle, 19000.0, 0.0002, (1, 200.0, 0.7),
                                                     (5, 1000.0, 0.0), (2, 20.0, 0.7)), x)
    check(out, lk, ref_out, ref_lk, "pilot PLL")


def test_pll_block_partition_and_state(sdr, oracle):
    rng = np.random.default_rng(4)
    nch, n = 5, 12345
    x = fm_channels(rng, nch, n)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    outs, lks, i = [], [], 0
    for step in (1, 7, 8, 9, 1000, 3):
        o, l = pll.process(x[:, i:i + step])
        outs.append(o)
        lks.append(l)
        i += step
    o, l = pll.process(x[:, i:])
    outs.append(o)
    lks.append(l)
    out, lk = np.concatenate(outs, axis=1), np.concatenate(lks, axis=1)
    whole = main_rs_design(sdr).design(RATE, nch=nch)
    wo, wl = whole.process(x)
    assert np.array_equal(out, wo) and np.array_equal(lk, wl)  # same per-sample arithmetic
    nph, val = pll.state(2)
    assert -1.0 < nph < 1.0 and abs(abs(val) - 1.0) < 1e-5
    c = pll.clone()
    o1, _ = pll.process(x[:, :100])
    o2, _ = c.process(x[:, :100])
    assert np.array_equal(o1, o2)


def test_pll_tone_kat(sdr):
    # steady tone at f -> output ~ f Hz and locked (examples/pll.rs expectation out ~ f)
    n, f0 = 40000, 50e3
    x = np.exp(2j * np.pi * f0 * np.arange(n) / RATE).astype(np.complex64)
    out, lk = main_rs_design(sdr).design(RATE).process(x)
    assert lk[20000:].all()
    assert abs(out[20000:].mean() - f0) < 0.01 * f0


def test_pll_apply_single_sample(sdr):
    pll = main_rs_design(sdr).design(RATE)
    assert pll.apply(1 + 0j) is None  # value starts at 0+0i -> c = 0 -> not locked


def test_pll_stereo_pilot_chain(sdr, oracle):
    """src/main.rs:56-69: 19 kHz pilot PLL on the 144 kHz FM audio, mono = v/2 and
    diff = (v / value.powi(2)).re / 2 while the pilot is locked -- bit-exact, batched."""
    f = sdr.filter
    rate = 144000.0
    rng = np.random.default_rng(19)
    nch, n = 6, 60000
    t = np.arange(n) / rate
    v = np.empty((nch, n), np.float32)
    for c in range(nch):
        lr = 0.3 * np.sin(2 * np.pi * 440 * t)
        lmr = 0.2 * np.sin(2 * np.pi * 1000 * t + c)
        ph = rng.uniform(-1.2, 1.2) if c < 4 else rng.uniform(2.0, 4.0)
        v[c] = (lr + 0.2 * np.cos(2 * np.pi * 19000 * t + ph)
                + lmr * np.cos(2 * np.pi * 38000 * t + 2 * ph)
                + 0.01 * rng.standard_normal(n)).astype(np.float32)
    design = f.PllDesign(19000.0, 0.0002, f.BiquadD.LowPass(200.0, 0.7),
                         f.BiquadD.LowPass(20.0, 0.7), f.BiquadD.LowPass(20.0, 0.7))
    pll = design.design(rate, nch=nch)
    mono, diff, locked = pll.stereo(v)
    op = oracle.pll_params(19000.0, 0.0002, rate, (1, 200.0, 0.7), (1, 20.0, 0.7),
                           (1, 20.0, 0.7))
    for c in range(nch):
        om, od, ol = oracle.pll_stereo(op, v[c])
        assert np.array_equal(mono[c], om)
        assert np.array_equal(locked[c], ol), c
        assert np.array_equal(diff[c], od), c
    assert locked.any() and diff[locked.astype(bool)].std() > 0
    # the normal output mode is restored afterwards and state carried on
    out2, _ = pll.process(v[:, :100].astype(np.complex64))
    assert out2.shape == (nch, 100)


def test_pll_rtl_tcp_u8_input(sdr, oracle):
    """src/main.rs:48-49: rtl.listen() feeds the PLL directly; u8 I/Q converted in the load
    ((v - 128) / 128, src/rtltcp.rs:156-164) gives exactly the C64 path's outputs."""
    rng = np.random.default_rng(23)
    nch, n = 70, 9001
    x = fm_channels(rng, nch, n)
    iq = np.empty((nch, 2 * n), np.uint8)
    iq[:, 0::2] = np.clip(np.round(x.real * 100 + 128), 0, 255)
    iq[:, 1::2] = np.clip(np.round(x.imag * 100 + 128), 0, 255)
    xc = oracle.u8_to_c64(iq.reshape(-1)).reshape(nch, n)
    d = main_rs_design(sdr)
    a = d.design(RATE, nch=nch)
    out_u8, lk_u8 = a.process_u8(iq[:, :4000])
    o2, l2 = a.process_u8(iq[:, 4000:])
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), xc)
    assert np.array_equal(np.concatenate([out_u8, o2], 1), ref_out)
    assert np.array_equal(np.concatenate([lk_u8, l2], 1), ref_lk)


def test_pll_examples_frequency_sweep_kat(sdr, oracle):
    """examples/pll.rs:8-18: the PLL over freq_sweep(1.8 MHz, df = 20 kHz, warmup,
    -200 kHz..200 kHz).  Bit-exact to the oracle, and the reference's expected picture: the
    loop locks over the middle of the sweep and its output tracks the input frequency, delayed
    by the output filter (LowPass 20 kHz: 24 samples at 4e8 Hz/s)."""
    rate = 1.8e6
    f, v = oracle.freq_sweep(rate, 20000.0, True, -200000.0, 200000.0)
    fl = sdr.filter
    d = fl.PllDesign(0.0, 0.035, fl.BiquadD.LowPass(80000.0, 0.7), fl.BiquadD.LowPass(20000.0, 0.7),
                     fl.BiquadD.LowPass(20000.0, 0.7))
    out, lk = d.design(rate).process(v)
    ro, rl = oracle.pll_batch(oracle_params(oracle, outf=(1, 20000.0, 0.7)), v)
    check(out, lk, ro[0], rl[0], "sweep")
    idx = np.nonzero(lk)[0]
    assert idx.size == idx[-1] - idx[0] + 1            # one contiguous locked stretch
    assert f[idx[0]] < -80000.0 and f[idx[-1]] > 80000.0
    delayed = f[idx - 24]
    assert np.abs(out[idx] - delayed).max() < 50.0     # out ~ f (24-sample filter delay)
    assert np.corrcoef(out[idx], f[idx])[0, 1] > 0.9999


@pytest.mark.parametrize("design", ["main", "examples"])
def test_pll_split_chain_helper_waves(sdr, oracle, design):
    """Output mode 0 on 64-channel-aligned banks with vector rows runs the chain on one wave
    and the lock / output filters + stores on a second (pll_split_kernel): two workgroups,
    device buffers with padded rows, a ragged tail (n % 8 != 0, whole steps after the LDS
    hand-back of the filter states) and a second call continuing the state; bit-exact."""
    from sdrgpu.device import DeviceBuffer
    f = sdr.filter
    rng = np.random.default_rng(31)
    nch, n1, n2, ld = 128, 12003, 4000, 16008
    x = fm_channels(rng, nch, n1 + n2)
    if design == "main":
        d, op = main_rs_design(sdr), oracle_params(oracle)
    else:
        d = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.BiquadD.LowPass(20000.0, 0.7),
                        f.BiquadD.LowPass(20000.0, 0.7))
        op = oracle_params(oracle, outf=(1, 20000.0, 0.7))
    pll = d.design(RATE, nch=nch)
    xp = np.zeros((nch, ld), np.complex64)
    outs, lks = [], []
    for a, b in ((0, n1), (n1, n1 + n2)):
        xp[:, :b - a] = x[:, a:b]
        dx = DeviceBuffer.from_numpy(xp)
        do = DeviceBuffer.empty(nch * ld, np.float32)
        dl = DeviceBuffer.empty(nch * ld, np.uint8)
        pll.process_dev(dx.ptr, ld, b - a, do.ptr, dl.ptr, ld)
        pll.sync()
        outs.append(do.download().reshape(nch, ld)[:, :b - a])
        lks.append(dl.download().reshape(nch, ld)[:, :b - a])
    ref_out, ref_lk = oracle.pll_batch(op, x, nthreads=8)
    check(np.concatenate(outs, 1), np.concatenate(lks, 1), ref_out, ref_lk, f"split {design}")


def special_operand_channels(rng, n):
    """One pathology per channel (so a NaN in one does not hide the others), each run through
    the loop long enough for the loop filter's output -- atan2f's operands, pll.rs:72 -- to
    reach it: exact zeros, subnormals, +-inf, NaN, huge / tiny magnitudes and ratios, signed
    zeros, exact +-1 (x == 1 in e_atan2f.c)."""
    base = fm_channels(rng, 1, n)[0]
    chans, names = [], []

    def add(name, x):
        names.append(name)
        chans.append(np.asarray(x, np.complex64))

    add("control", base)
    z = base.copy()
    z[1000:4000] = 0                     # loop biquad decays through subnormals to exact 0
    add("zero burst", z)
    add("all zeros", np.zeros(n, np.complex64))
    nz = np.full(n, complex(-0.0, -0.0), np.complex64)
    add("negative zeros", nz)
    add("subnormal 1e-39", base * np.float32(1e-39))
    add("subnormal 1e-44", base * np.float32(1e-44))
    sb = base.copy()
    sb[2000:2600] *= np.float32(1e-41)   # a subnormal burst inside a locked stream
    add("subnormal burst", sb)
    for name, pos, val in (("+inf re", 2000, complex(np.inf, 0)),
                           ("-inf im", 2000, complex(0, -np.inf)),
                           ("nan", 2000, complex(np.nan, 1.0))):
        x = base.copy()
        x[pos] = val
        add(name, x)
    add("huge 1e30", base * np.float32(1e30))
    with np.errstate(over="ignore"):
        add("overflow 3e38", base * np.float32(3e38))
    add("tiny 1e-30", base * np.float32(1e-30))
    add("re huge / im tiny",
        (base.real * np.float32(1e30)) + 1j * (base.imag * np.float32(1e-30)))
    add("re tiny / im huge",
        (base.real * np.float32(1e-30)) + 1j * (base.imag * np.float32(1e30)))
    pm = np.where(rng.random(n) < 0.5, 1.0, -1.0).astype(np.float32)
    add("exact +-1 real", pm.astype(np.complex64))
    add("exact 1", np.ones(n, np.complex64))
    return np.stack(chans), names


def test_pll_special_operands_bit_exact(sdr, oracle):
    """Pll::apply (src/filter/pll.rs:70-85) fed the operands that reach atan2f's special-case
    path (the branch-free selects and their wave ballot, csrc/libm_glibc.h) and the subnormal
    / overflow ranges of the loop filter: outputs and lock flags equal the oracle's bit for
    bit (NaN-aware: NaN where the oracle has NaN), on both kernel forms (the split
    chain/helper kernel on 16-B aligned rows, the single-wave kernel on an odd row pitch)."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(77)
    n = 6000
    x, names = special_operand_channels(rng, n)
    nch = x.shape[0]
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), x, nthreads=8)
    for ld in (n, n + 1):
        pll = main_rs_design(sdr).design(RATE, nch=nch)
        xp = np.zeros((nch, ld), np.complex64)
        xp[:, :n] = x
        dx = DeviceBuffer.from_numpy(xp)
        do = DeviceBuffer.empty(nch * ld, np.float32)
        dl = DeviceBuffer.empty(nch * ld, np.uint8)
        pll.process_dev(dx.ptr, ld, n, do.ptr, dl.ptr, ld)
        pll.sync()
        out = do.download().reshape(nch, ld)[:, :n]
        lk = dl.download().reshape(nch, ld)[:, :n]
        for c, name in enumerate(names):
            assert np.array_equal(lk[c], ref_lk[c]), f"ld={ld} {name}: lock flags differ"
            g, r = out[c].view(np.uint32), ref_out[c].view(np.uint32)
            bad = (g != r) & ~(np.isnan(out[c]) & np.isnan(ref_out[c]))
            assert not bad.any(), (f"ld={ld} {name}: {bad.sum()} outputs differ, first at "
                                   f"{np.flatnonzero(bad)[0]}")


# ---- time-parallel blocks (pll.hip "speculative segments"): bit-identical to the serial PLL ----

@pytest.mark.parametrize("seg,warm", [(4096, 4096), (2048, 64), (8192, 16384), (1000, 512)],
                         ids=["converging", "mostly-recomputed", "warm-reaches-start", "ragged"])
def test_pll_time_parallel_bit_exact(sdr, oracle, seg, warm):
    """main.rs PLL (src/main.rs:41-46; src/filter/pll.rs:70-85) over 96 FM channels with each
    block cut into concurrent segments: with a warm-up long enough for most segments to reach
    the true state (converging), one so short that almost every segment is recomputed from the
    true state, one reaching back to sample 0, and a segment length that is not a multiple of
    8 (rounded up) with a ragged last segment.  Outputs and lock flags array_equal to the oracle
    (the serial reference), over two calls (state carried) and against the serial kernel."""
    rng = np.random.default_rng(700 + seg + warm)
    nch, n = 96, 30011
    x = fm_channels(rng, nch, n)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    pll.set_time_parallel(seg, warm)
    s_plan, w_plan = pll.time_parallel_plan(20000)
    assert s_plan == (seg + 7) // 8 * 8 and w_plan == warm
    o1, l1 = pll.process(x[:, :20000])
    segs, rec = pll.last_time_parallel()
    assert segs == -(-20000 // s_plan) and 0 <= rec <= nch * (segs - 1)
    if warm >= 20000 - s_plan:      # every warm-up reaches back to sample 0: exact by construction
        assert rec == 0
    if warm == 64:                  # far too short to converge: the fix path carries the block
        assert rec > nch
    o2, l2 = pll.process(x[:, 20000:])
    out, lk = np.concatenate([o1, o2], axis=1), np.concatenate([l1, l2], axis=1)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), x, nthreads=16)
    check(out, lk, ref_out, ref_lk, f"time-parallel seg {seg} warm {warm}")
    serial = main_rs_design(sdr).design(RATE, nch=nch)
    serial.set_time_parallel(-1)
    assert serial.time_parallel_plan(n) == (0, 4096)
    so, sl = serial.process(x)
    assert np.array_equal(so, out) and np.array_equal(sl, lk)
    # the carried state is the serial one too: one more block agrees
    a, b = pll.process(x[:, :3000]), serial.process(x[:, :3000])
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_pll_time_parallel_other_designs_and_u8(sdr, oracle):
    """examples/pll.rs's design (output LowPass: an output-filter state in the segments'
    state), the stereo pilot's output mode (src/main.rs:55-66) and rtl_tcp u8 input, each with
    forced segments: bit-exact to the oracle / to the serial handle."""
    f = sdr.filter
    rng = np.random.default_rng(77)
    nch, n = 40, 24000
    x = fm_channels(rng, nch, n)
    d = f.PllDesign(0.0, 0.035, f.BiquadD.LowPass(80000.0, 0.7), f.BiquadD.LowPass(20000.0, 0.7),
                    f.BiquadD.LowPass(20000.0, 0.7))
    pll = d.design(RATE, nch=nch)
    pll.set_time_parallel(3000, 2048)
    out, lk = pll.process(x)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle, outf=(1, 20000.0, 0.7)), x, nthreads=16)
    check(out, lk, ref_out, ref_lk, "examples/pll.rs design, time-parallel")
    iq = rng.integers(0, 256, size=(nch, 2 * n), dtype=np.uint8)
    a = main_rs_design(sdr).design(RATE, nch=nch)
    a.set_time_parallel(4000, 4000)
    b = main_rs_design(sdr).design(RATE, nch=nch)
    b.set_time_parallel(-1)
    oa, la = a.process_u8(iq)
    ob, lb = b.process_u8(iq)
    assert np.array_equal(oa, ob) and np.array_equal(la, lb)
    t = np.arange(n) / 144e3
    v = (0.3 * np.cos(2 * np.pi * 19000.0 * t[None, :] + rng.uniform(0, 6, (4, 1)))).astype(np.float32)
    pd = f.PllDesign(19000.0, 0.0002, f.BiquadD.LowPass(200.0, 0.7), f.BiquadD.LowPass(20.0, 0.7),
                     f.BiquadD.LowPass(20.0, 0.7))
    p1, p2 = pd.design(144e3, nch=4), pd.design(144e3, nch=4)
    p1.set_time_parallel(2048, 1024)
    p2.set_time_parallel(-1)
    m1, d1, k1 = p1.stereo(v)
    m2, d2, k2 = p2.stereo(v)
    assert np.array_equal(d1, d2) and np.array_equal(k1, k2)


def test_pll_time_parallel_auto_plan_configs3(sdr, oracle):
    """The automatic plan at configs[3]'s shape (1024 channels x 2^20: 64 segments of 16 Ki,
    4 Ki of warm-up, one wave per SIMD), and a 1024-channel block of 2^17 samples through it
    (auto plan: 32 segments of 4 Ki) array_equal to the oracle on 8 channels."""
    nch = 1024
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    assert pll.time_parallel_plan(1 << 20) == (16384, 4096)
    assert pll.time_parallel_plan(8191) == (0, 4096)       # under two segments: serial
    rng = np.random.default_rng(1024)
    n = 1 << 17
    chans = [0, 63, 64, 511, 777, 1000, 1022, 1023]
    x = np.empty((nch, n), np.complex64)
    x[:] = fm_channels(rng, 1, n)[0]                           # one waveform everywhere ...
    x[chans] = fm_channels(rng, len(chans), n)                 # ... and 8 different channels
    assert pll.time_parallel_plan(n) == (4096, 4096)
    out, lk = pll.process(x)
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), np.ascontiguousarray(x[chans]), nthreads=8)
    check(out[chans], lk[chans], ref_out, ref_lk, "configs[3] auto plan")
    assert np.array_equal(out[1], out[2]) and np.array_equal(out[1], out[1020])


def test_pll_in_place_long_block(sdr, oracle):
    """process_dev with the f32 outputs written over the c64 input rows (d_out = d_in,
    ld_out = 2 ld_in: each output row inside its own input row) on a block the automatic plan
    would cut into segments: the handle runs its serial pass (the segment kernels re-read inputs
    after outputs are stored), so outputs and lock flags stay array_equal to the oracle
    (src/filter/pll.rs:70-85), over two blocks with the state carried."""
    from sdrgpu.device import DeviceBuffer
    rng = np.random.default_rng(79)
    nch, n = 64, 1 << 15
    x = fm_channels(rng, nch, 2 * n)
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    assert pll.time_parallel_plan(n)[0] > 0
    outs, lks = [], []
    for h in range(2):
        dx = DeviceBuffer.from_numpy(np.ascontiguousarray(x[:, h * n:(h + 1) * n]))
        dl = DeviceBuffer.empty(nch * 2 * n, np.uint8)  # lock rows share ld_out = 2 n
        pll.process_dev(dx.ptr, n, n, dx.ptr, dl.ptr, 2 * n)
        pll.sync()
        assert pll.last_time_parallel()[0] == 0  # serial pass
        outs.append(dx.download(nch * 2 * n, np.float32).reshape(nch, 2 * n)[:, :n])
        lks.append(dl.download(dtype=np.uint8).reshape(nch, 2 * n)[:, :n])
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), x, nthreads=16)
    check(np.concatenate(outs, axis=1), np.concatenate(lks, axis=1), ref_out, ref_lk, "in place")


def test_pll_time_parallel_adapts_to_misses(sdr, oracle):
    """The automatic plan adapts per handle (src/filter/pll.rs:70-85 is serial; this is the
    speculation's fallback): with an 8-sample warm-up nearly every segment's guess misses, so the
    block runs pass 1, the re-run pass and the walk; the handle then runs the next 8 blocks as one
    serial pass each and probes segments again -- plan sequence (tp, 8 x serial, tp) -- while
    every output stays array_equal to the oracle; reset() starts the adaptation over.  (On
    unlocked noise the default 4 Ki warm-up still meets most true states: 58 of 256 segments
    missed on the GPU, so the default plan keeps running segments there.)"""
    rng = np.random.default_rng(80)
    nch, n, blocks = 64, 1 << 14, 10
    pll = main_rs_design(sdr).design(RATE, nch=nch)
    pll.set_time_parallel(0, 8)     # automatic segments, 8 samples of warm-up
    assert pll.time_parallel_plan(n) == (4096, 8)
    x = fm_channels(rng, nch, n * blocks)
    outs, lks, plan = [], [], []
    for b in range(blocks):
        o, lk = pll.process(x[:, b * n:(b + 1) * n])
        plan.append(pll.last_time_parallel())
        outs.append(o)
        lks.append(lk)
    assert plan[0][0] > 0 and 2 * plan[0][1] > plan[0][0] * nch, plan[0]
    assert all(p[0] == 0 for p in plan[1:9]), plan
    assert plan[9][0] > 0, plan
    ref_out, ref_lk = oracle.pll_batch(oracle_params(oracle), x, nthreads=16)
    check(np.concatenate(outs, axis=1), np.concatenate(lks, axis=1), ref_out, ref_lk, "adapted plan")
    pll.process(x[:, :n])
    assert pll.last_time_parallel()[0] == 0     # inside the serial stretch again
    pll.reset()
    pll.process(x[:, :n])
    assert pll.last_time_parallel()[0] > 0
