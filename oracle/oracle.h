/*
 * oracle.h -- CPU restatement of the agrif/unnamed-rust-sdr sample-stream hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the sdrgpu HIP
 * path and the timed CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path (libsdrgpu.so) never
 * links or calls it.
 *
 * Parity status: the reference crate (Rust) cannot be built here (no cargo/rustc, no
 * network) and ships no tests, fixtures or golden vectors.
 * The restatement is therefore cross-checked against independent float64
 * implementations (SciPy lfilter / NumPy FFT) and known-answer tests derived from the
 * reference examples (tests/golden/make_golden.py).  "parity unpinned" against reference
 * outputs; see DESIGN.md section "Oracle".
 *
 * Arithmetic contract (matches Rust defaults on x86-64 Linux): f32 everywhere, no FMA
 * contraction (-ffp-contract=off), sequential accumulation order exactly as written in
 * the reference, glibc libm sinf/cosf/atan2f/expf (what Rust std's f32 methods call).
 */
#ifndef SDR_ORACLE_H
#define SDR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_F32 = 0, ORACLE_C64 = 1 };

/* ---------------- FIR (src/filter/fir.rs:6-58, convolve.rs:4-16) ------------------
 * Streaming FIR with the reference's zero-initialised history and sequential MAC order,
 * followed by the Decimate adapter (src/signal/adapters/mod.rs:13-41): with decim D the
 * kept outputs are stream indices D-1, 2D-1, ...  All outputs are computed (as the
 * reference does), the dropped ones are discarded. */
typedef struct oracle_fir oracle_fir;
oracle_fir* oracle_fir_create(int sample_kind, int tap_kind, const float* taps,
                              size_t ntaps, uint32_t decim);
void   oracle_fir_destroy(oracle_fir* f);
void   oracle_fir_reset(oracle_fir* f);
/* in: n_in samples (f32 or interleaved re,im); out: kept outputs. Returns count. */
size_t oracle_fir_process(oracle_fir* f, const float* in, size_t n_in, float* out);
/* Batched helper: nch independent channels (channel-major, leading dims in samples). */
size_t oracle_fir_batch(int sample_kind, int tap_kind, const float* taps, size_t ntaps,
                        uint32_t decim, size_t nch, const float* in, size_t ld_in,
                        size_t n_in, float* out, size_t ld_out, int nthreads);

/* ---------------- Biquad (src/filter/biquad.rs:4-155) ---------------------------- */
enum {
    ORACLE_BQ_IDENTITY = 0, /* filter::Identity, src/filter/simple.rs:3-19 */
    ORACLE_BQ_LOWPASS = 1,
    ORACLE_BQ_HIGHPASS = 2,
    ORACLE_BQ_BANDPASS = 3,
    ORACLE_BQ_NOTCH = 4,
    ORACLE_BQ_LR = 5,
};
typedef struct { int kind; float freq; float q; } oracle_biquad_design;
/* normalised coefficients b0,b1,b2,na1,na2 as Biquad::new computes them (:25-38) */
typedef struct { float b0, b1, b2, na1, na2; } oracle_biquad_coefs;
void oracle_biquad_design_coefs(oracle_biquad_design d, float rate, oracle_biquad_coefs* c);
/* Run a biquad over a real or complex stream from zero state (biquad.rs:42-56). */
void oracle_biquad_run(oracle_biquad_design d, float rate, int sample_kind,
                       const float* in, size_t n, float* out);

/* ---------------- PLL (src/filter/pll.rs:3-86) ----------------------------------- */
typedef struct {
    float reference;               /* Hz, divided by rate at design (pll.rs:51) */
    float gain;                    /* pll.rs:52 */
    float rate;                    /* stream rate (FilterDesign::design(rate)) */
    oracle_biquad_design loopf;    /* Complex<f32> filter */
    oracle_biquad_design outputf;  /* f32 filter (Identity allowed) */
    oracle_biquad_design lockf;    /* f32 filter */
} oracle_pll_params;
/* Process nch channels x n samples (channel-major c64).  out[ch*ld_out+i] is the
 * output when locked else 0.0 (src/main.rs:49 unwrap_or(0.0)); locked[] is 1/0. */
void oracle_pll_batch(const oracle_pll_params* p, size_t nch, const float* in,
                      size_t ld_in, size_t n, float* out, uint8_t* locked,
                      size_t ld_out, int nthreads);

/* FM stereo pilot map (src/main.rs:56-69) on one real stream: mono, diff, lock mask. */
void oracle_pll_stereo(const oracle_pll_params* p, const float* v, size_t n, float* mono,
                       float* diff, uint8_t* locked);

/* ---------------- FFT (src/fft.rs:3-37) ------------------------------------------ */
/* fft::fft on one frame of n complex samples: forward DFT (computed in float64,
 * rounded to f32 -- rustfft 3.0 itself is unpinned), fftshift-collated,
 * multiplied by norm = 1/sqrt(n) in f32 (fft.rs:14-26). */
void oracle_fft_frame(const float* in, size_t n, float* out);
/* Window(n) + Decimate(hop) framing (src/signal/adapters/mod.rs:270-303, 13-41) over a
 * whole stream, frame j = x[(j+1)hop-n .. (j+1)hop-1] with zeros before the start, each
 * frame through oracle_fft_frame.  Returns the number of frames (n_in / hop). */
size_t oracle_stft(const float* in, size_t n_in, size_t n, size_t hop, float* out,
                   size_t max_frames, int nthreads);

/* ---------------- Sample-rate conversion (src/resample.rs:32-110) ----------------
 * libsamplerate (libsamplerate-sys, a git dependency, Cargo.toml:24-26; not in this image,
 * version unpinned) restated from its published src_zoh.c / src_linear.c / samplerate.c:
 * src_new + src_process (argument checks, last_ratio priming) + the converter's process
 * loop (f64 position walk, f32 samples, last_value carried across calls), src_reset,
 * src_set_ratio.  Converter ids: 0..2 = sinc (below), 3 = ZERO_ORDER_HOLD, 4 = LINEAR.
 * Parity unpinned: no libsamplerate outputs are available here. */
typedef struct oracle_src oracle_src;
oracle_src* oracle_src_new(int converter, int channels, int* error);
void oracle_src_delete(oracle_src* s);
int  oracle_src_reset(oracle_src* s);
int  oracle_src_set_ratio(oracle_src* s, double ratio);
/* SRC_DATA's fields as arguments; returns the libsamplerate error code */
int  oracle_src_process(oracle_src* s, const float* in, long in_frames, float* out,
                        long out_frames, double ratio, long* in_used, long* out_gen);

/* Sinc converters 0 / 1 / 2 (Best / Medium / Fastest) follow libsamplerate 0.2's src_sinc.c
 * with our own Kaiser-windowed sinc tables of libsamplerate's increments and lengths (its
 * coefficient headers are absent): parity unpinned.  oracle_sinc_table writes the table
 * (returns its length; out == NULL asks for the length only) and its increment. */
int  oracle_sinc_table(int converter, float* out, int cap, int* increment);

/* ---------------- Sources (src/signal/sources.rs) ------------------------------- */
/* freq(rate, f, phase) (sources.rs:196-221 via FreqSweep::next :150-175), n samples */
void oracle_freq(float rate, float freq, float phase, size_t n, float* out);
/* freq_sweep(rate, df, warmup, start..end) (sources.rs:181-194 via FreqSweep, :116-179):
 * up to cap (freq, value) samples; returns the sweep length */
size_t oracle_freq_sweep(float rate, float df, int warmup, float start, float end, size_t cap,
                         float* freqs, float* out);
/* rtl_tcp u8 IQ -> f32 (src/rtltcp.rs:156-164) */
void oracle_u8_to_c64(const uint8_t* in, size_t n, float* out);

/* glibc atan2f (fn 0: out0 = atan2f(a, b)) or sinf / cosf (fn 1: out0 = sinf(a), out1 =
 * cosf(a)) -- what num-complex's arg() / from_polar call through Rust std in Pll::apply
 * (src/filter/pll.rs:72-76); the reference for sdrgpu_debug_libm. */
void oracle_libm(int fn, const float* a, const float* b, float* out0, float* out1, size_t n);

#ifdef __cplusplus
}
#endif
#endif
