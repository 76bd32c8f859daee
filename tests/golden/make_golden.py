"""Generate the golden fixtures in tests/golden/ (committed; re-run to regenerate).

The reference crate (Rust) cannot be built or run in this environment and ships no
tests or vectors.  These fixtures are therefore computed from
INDEPENDENT float64 implementations (SciPy lfilter, NumPy FFT) and closed-form known
answers derived from the reference examples -- never from the oracle or the GPU code.
Inputs are seeded; each fixture is a small .npz (no pickles).

  fir_c1.npz      127-tap real FIR over real samples (configs[0] shape, shortened)
  fir_c2.npz      255-tap real taps, complex IQ, decimate 4 (configs[1] shape, shortened)
  fir_cc.npz      63-tap complex taps, complex IQ, decimate 3
  biquad.npz      RBJ designs (biquad.rs:83-155) in float64 + impulse responses
  fft.npz         fft::fft (fft.rs:3-28) of random frames, fftshift / sqrt(N)
  stft.npz        Window+Decimate framing (adapters/mod.rs:270-303) + fft per frame
  resample.npz    libsamplerate ZOH / linear (src/resample.rs) from the closed form with
                  exact rational positions q_k = k / ratio - 1 (x[-1] = x[0] after reset),
                  not the serial f64 walk the oracle restates
  fft_any.npz     fft::fft / rfft at lengths that are not powers of two (rustfft plans any
                  N, src/fft.rs:10-11): the reference's own callers' 1000-point window
                  (examples/live.rs:30) and 14,400-point rfft (examples/fft.rs:64,78 at
                  144 kHz), plus 1001 = 7*11*13, primes 17 / 1009 / 4099, 6, 12288; and a
                  1000-point STFT (Window + Decimate) over a short stream
"""
from fractions import Fraction
import os

import numpy as np
import scipy.signal as ss

HERE = os.path.dirname(os.path.abspath(__file__))


def cplx(rng, n):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)


def fir_ref(h, x, decim):
    y = ss.lfilter(h.astype(np.complex128 if np.iscomplexobj(h) else np.float64), [1.0],
                   x.astype(np.complex128 if np.iscomplexobj(x) else np.float64))
    return y[decim - 1::decim]


def main():
    rng = np.random.default_rng(20240601)
    # configs[0]: 127-tap real lowpass FIR over f32 samples
    h1 = ss.firwin(127, 0.2).astype(np.float32)
    x1 = rng.standard_normal(4096).astype(np.float32)
    np.savez(os.path.join(HERE, "fir_c1.npz"), taps=h1, x=x1, decim=1, y=fir_ref(h1, x1, 1))
    # configs[1]: 255-tap FIR, complex IQ, decimate by 4
    h2 = ss.firwin(255, 0.2).astype(np.float32)
    x2 = cplx(rng, 8192)
    np.savez(os.path.join(HERE, "fir_c2.npz"), taps=h2, x=x2, decim=4, y=fir_ref(h2, x2, 4))
    # complex taps (Complex * Complex MAC, convolve.rs:13-15)
    n = np.arange(63)
    h3 = (ss.firwin(63, 0.3) * np.exp(0.7j * n)).astype(np.complex64)
    x3 = cplx(rng, 3000)
    np.savez(os.path.join(HERE, "fir_cc.npz"), taps=h3, x=x3, decim=3, y=fir_ref(h3, x3, 3))

    # Biquad designs in float64 (RBJ cookbook exactly as biquad.rs:89-151 writes them)
    rate = 1.8e6
    designs = [(1, 80000.0, 0.7), (2, 20000.0, 0.7), (3, 19000.0, 2.0), (4, 50000.0, 1.0),
               (5, 13333.0, 0.0)]
    coefs, imp = [], []
    for kind, f, q in designs:
        if kind == 5:
            decayn = f / rate
            a = [1.0, -np.exp(-decayn), 0.0]
            b = [decayn, 0.0, 0.0]
        else:
            w = 2 * np.pi * f / rate
            c, s = np.cos(w), np.sin(w)
            al = s / (2 * q)
            a = [1 + al, -2 * c, 1 - al]
            b = {1: [(1 - c) / 2, 1 - c, (1 - c) / 2], 2: [(1 + c) / 2, -1 - c, (1 + c) / 2],
                 3: [al, 0.0, -al], 4: [1.0, -2 * c, 1.0]}[kind]
        nb = [bb / a[0] for bb in b]
        coefs.append(nb + [-a[1] / a[0], -a[2] / a[0]])
        d = np.zeros(256)
        d[0] = 1.0
        imp.append(ss.lfilter(nb, [1.0, a[1] / a[0], a[2] / a[0]], d))
    np.savez(os.path.join(HERE, "biquad.npz"), designs=np.array(designs), rate=rate,
             coefs=np.array(coefs), impulse=np.array(imp))

    # fft::fft: out[i] = X[(i - N/2) mod N] / sqrt(N)
    frames = {}
    for N in (8, 64, 1024, 4096):
        xf = cplx(rng, N)
        frames[f"x{N}"] = xf
        frames[f"y{N}"] = np.fft.fftshift(np.fft.fft(xf.astype(np.complex128))) / np.sqrt(N)
    np.savez(os.path.join(HERE, "fft.npz"), **frames)

    # STFT: window(n) + decimate(hop); frame j = x[(j+1)hop-n, (j+1)hop), zeros before 0
    N, hop = 64, 32
    xs = cplx(rng, 32 * 10 + 5)
    nf = xs.size // hop
    Y = np.zeros((nf, N), np.complex128)
    for j in range(nf):
        beg = (j + 1) * hop - N
        fr = np.zeros(N, np.complex128)
        for i in range(N):
            if beg + i >= 0:
                fr[i] = xs[beg + i]
        Y[j] = np.fft.fftshift(np.fft.fft(fr)) / np.sqrt(N)
    np.savez(os.path.join(HERE, "stft.npz"), x=xs, n=N, hop=hop, y=Y)

    # resampler: ratios of src/main.rs (1.8 Msps -> 144 kHz -> 48 kHz) and generic ones
    cases = {}
    for ci, (ratio, ch) in enumerate([(144000 / 1.8e6, 1), (48000 / 144000, 2), (1.37, 1),
                                      (3.0, 2), (48000 / 44100, 1)]):
        xr = rng.standard_normal((2000, ch)).astype(np.float32)
        cases[f"x{ci}"] = xr
        cases[f"ratio{ci}"] = np.float64(ratio)
        cases[f"lin{ci}"], cases[f"linamb{ci}"] = src_closed_form(xr, ratio, True)
        cases[f"zoh{ci}"], cases[f"zohamb{ci}"] = src_closed_form(xr, ratio, False)
    np.savez(os.path.join(HERE, "resample.npz"), ncases=5, **cases)

    # any-N fft::fft (numpy fftshift rolls by N // 2 = the reference's -(N/2) start, odd N too)
    anyn = {}
    sizes = (6, 17, 1000, 1001, 1009, 4099, 12288, 14400)
    for N in sizes:
        xf = cplx(rng, N)
        anyn[f"x{N}"] = xf
        anyn[f"y{N}"] = np.fft.fftshift(np.fft.fft(xf.astype(np.complex128))) / np.sqrt(N)
    # rfft (fft.rs:30-37): collated output with the first N/2 entries drained
    for N in (1001, 14400):
        xr = rng.standard_normal(N).astype(np.float32)
        full = np.fft.fftshift(np.fft.fft(xr.astype(np.complex128))) / np.sqrt(N)
        anyn[f"rx{N}"] = xr
        anyn[f"ry{N}"] = full[N // 2:]
    # 1000-point STFT, hop 300 (live.rs window(1000/rate).decimate(fps))
    N, hop = 1000, 300
    xs = cplx(rng, 3000 + 77)
    nf = xs.size // hop
    Y = np.zeros((nf, N), np.complex128)
    for j in range(nf):
        beg = (j + 1) * hop - N
        fr = np.zeros(N, np.complex128)
        lo = max(0, beg)
        fr[lo - beg:] = xs[lo:beg + N]
        Y[j] = np.fft.fftshift(np.fft.fft(fr)) / np.sqrt(N)
    anyn.update(sx=xs, sn=N, shop=hop, sy=Y)
    np.savez(os.path.join(HERE, "fft_any.npz"), sizes=np.array(sizes), **anyn)


def src_closed_form(x, ratio, linear):
    """One src_process call after reset at constant ratio, whole input, unlimited output:
    output k sits at exact position q = k * inc - 1 (inc = the f64 1/ratio) between frames
    floor(q) and floor(q)+1, frame -1 being last_value = x[0]; linear needs the right frame
    (q < N - 1), ZOH holds the left one (q <= N - 1)."""
    n = x.shape[0]
    inc = Fraction(1.0 / ratio)
    out, amb = [], []
    k = 0
    while True:
        q = k * inc - 1
        fl = q.numerator // q.denominator
        if (linear and not q < n - 1) or (not linear and not q <= n - 1):
            break
        fr = float(q - fl)
        amb.append(min(fr, 1 - fr) < 1e-9)  # the serial f64 walk may land on either side
        a = x[max(fl, 0)].astype(np.float64)
        if linear:
            b = x[fl + 1].astype(np.float64)
            f = float(q - fl)
            out.append((a + f * (b - a)).astype(np.float32))
        else:
            out.append(a.astype(np.float32))
        k += 1
    return np.array(out, np.float32).reshape(-1, x.shape[1]), np.array(amb, bool)


if __name__ == "__main__":
    main()
