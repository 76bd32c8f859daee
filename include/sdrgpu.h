/*
 * sdrgpu.h -- C ABI of the MI355X-native sample-stream core (FIR / FIR-decimate,
 * framed FFT / STFT, batched PLL) that replaces the CPU hot path of the Rust crate
 * agrif/unnamed-rust-sdr (`sdr` 0.1.0).
 *
 * Every entry point names the reference interface it replaces (path:line in the
 * reference tree).  The ABI is modelled on the crate's only existing FFI boundary,
 * src/resample.rs (libsamplerate-sys):
 *   - opaque handle per filter, create/clone/reset/destroy
 *     (SampleRate::new / try_clone / reset / Drop, src/resample.rs:32-110);
 *   - int error codes, 0 = OK, positive = named error, sdrgpu_strerror()
 *     (resample::Error, src/resample.rs:151-270);
 *   - block-oriented process() (SampleRate::process, src/resample.rs:46-67) -- a
 *     per-sample FFI call would be infeasible, so the Rust side buffers samples.
 *
 * Threading: a handle is Send, not Sync (the Block adapter moves filters across rayon
 * workers, src/signal/adapters/block.rs:142-146).  Calls on one handle must not run
 * concurrently; a handle may migrate between threads.  Each handle owns one HIP stream
 * (or uses one set with *_set_stream).
 *
 * Buffers: the plain functions take HOST pointers and are synchronous.  The *_dev
 * variants take DEVICE pointers (on the handle's device), enqueue on the handle's stream
 * and return immediately; call *_sync or synchronise the stream before reading.
 *
 * Sample layout: SDRGPU_F32 = float; SDRGPU_C64 = {float re, im} interleaved, i.e.
 * num::Complex<f32> (#[repr(C)]).  Sizes are counted in SAMPLES, not bytes.
 */
#ifndef SDRGPU_H
#define SDRGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDRGPU_ABI_VERSION 1

/* ---- error codes (style of resample::Error, src/resample.rs:151-270) ---- */
enum sdrgpu_status {
    SDRGPU_OK = 0,
    SDRGPU_ERR_INVALID = 1,      /* null handle/pointer, zero taps, zero decimation, bad kind */
    SDRGPU_ERR_NOMEM = 2,        /* host or device allocation failed */
    SDRGPU_ERR_DEVICE = 3,       /* HIP runtime error (copy, stream, sync) */
    SDRGPU_ERR_NODEVICE = 4,     /* no GPU, or device index out of range */
    SDRGPU_ERR_UNSUPPORTED = 5,  /* valid request this build does not implement */
    SDRGPU_ERR_OUTPUT_CAP = 6,   /* output capacity smaller than the samples produced */
    SDRGPU_ERR_LAUNCH = 7,       /* kernel launch failed */
};

enum sdrgpu_kind {
    SDRGPU_F32 = 0,  /* f32 */
    SDRGPU_C64 = 1,  /* num::Complex<f32> */
    SDRGPU_CU8 = 2,  /* FIR input only: interleaved u8 I/Q as read from rtl_tcp
                        (RtlTcpConnection::read, src/rtltcp.rs:136-140), converted to
                        Complex<f32> as RtlTcpSignal::next does, (v - 128) / 128
                        (src/rtltcp.rs:156-164), inside the FIR load; outputs are C64.
                        1 sample = 2 bytes. */
};

/* FIR algorithm selection (results agree within the parity tolerance). */
enum sdrgpu_fir_algo {
    SDRGPU_FIR_AUTO = 0,          /* pick per shape */
    SDRGPU_FIR_DIRECT = 1,        /* LDS-tiled direct form, register-blocked outputs */
    SDRGPU_FIR_OVERLAP_SAVE = 2,  /* polyphase overlap-save, LDS-resident FFT tiles */
    SDRGPU_FIR_MATRIX = 3,        /* direct form on the matrix cores with an f32-accurate operand
                                     split: per-tile scaled fp16 x2 (c64, decim 1/2/4, ntaps up
                                     to 257; rtl_tcp u8 on int8 digits) or exact bf16 x3 (c64,
                                     decim 8); f32 taps, 16-B aligned c64 input.  AUTO picks it
                                     for those shapes.  The fp16 split is block floating point:
                                     a sample more than 2^29 below the largest sample of its
                                     1024-sample tile is resolved to 2^-38 of that sample, not
                                     to its own level (DIRECT keeps f32's range per sample). */
};

/* Which kernel ran the most recent block (sdrgpu_fir_last_kernel; test / bench introspection,
 * no reference counterpart).  The CU8 bit is set when rtl_tcp u8 input was first converted to
 * c64 by its own launch (shapes and alignments the fused u8 kernels do not take). */
enum sdrgpu_fir_kernel {
    SDRGPU_FIR_KERNEL_NONE = 0,
    SDRGPU_FIR_KERNEL_FP16 = 1,          /* fir_mxh: LDS-staged per-tile scaled fp16 x2 MFMA */
    SDRGPU_FIR_KERNEL_INT8 = 2,          /* fir_mxi: rtl_tcp u8 on the int8 MFMAs (16-B aligned) */
    SDRGPU_FIR_KERNEL_BF16X3 = 3,        /* fir_mfma: register-fed exact bf16 x3 MFMA */
    SDRGPU_FIR_KERNEL_OVERLAP_SAVE = 4,
    SDRGPU_FIR_KERNEL_DIRECT = 5,
    SDRGPU_FIR_KERNEL_CU8_CONVERTED = 16  /* flag */
};

const char* sdrgpu_strerror(int code);   /* resample::Error Display, src/resample.rs:209-269 */
int sdrgpu_abi_version(void);
int sdrgpu_device_count(int* count);

/* ---- device memory, streams and timing ----
 * The _dev entry points need device buffers; these helpers let a host without its own
 * GPU runtime (the Rust crate, C callers, the Python mirror) allocate them.  No reference
 * counterpart: the reference is CPU-only.  kind: 0 H2D, 1 D2H, 2 D2D. */
enum sdrgpu_copy_kind { SDRGPU_H2D = 0, SDRGPU_D2H = 1, SDRGPU_D2D = 2 };
int sdrgpu_dev_alloc(int device, size_t bytes, void** dptr);
int sdrgpu_dev_free(int device, void* dptr);
/* Pinned (page-locked) host memory for the *_async entry points: copies from/to it are DMA
 * straight from the caller's buffer and do not block the calling thread. */
int sdrgpu_host_alloc(int device, size_t bytes, void** hptr);
int sdrgpu_host_free(void* hptr);
int sdrgpu_dev_copy(int device, void* dst, const void* src, size_t bytes, int kind);
int sdrgpu_dev_memset(int device, void* dptr, int value, size_t bytes);
int sdrgpu_dev_synchronize(int device);
/* HIP events for timing work enqueued on a handle's stream (see *_get_stream). */
int sdrgpu_event_create(int device, void** event);
int sdrgpu_event_record(void* event, void* hip_stream);
int sdrgpu_event_synchronize(void* event);
int sdrgpu_event_elapsed_ms(void* start, void* end, float* ms);
int sdrgpu_event_destroy(void* event);

/* =====================================================================================
 * FIR / FIR-decimate.
 * Replaces: Fir::new / Fir::apply            (src/filter/fir.rs:12-32)
 *           Convolve::accumulate (MAC)       (src/filter/convolve.rs:8-15)
 *           FilterDesign for Fir/Vec<C>/&[C] (src/filter/fir.rs:36-58)
 *           Signal::filter + adapters::Filter::next (src/signal/mod.rs:42-48,
 *                                            src/signal/adapters/mod.rs:77-96)
 *           Signal::decimate + Decimate::next (src/signal/mod.rs:26-28,
 *                                            src/signal/adapters/mod.rs:19-37)
 * y[n] = sum_{k<ntaps} taps[k] * x[n-k], x[<0] = 0 (zero history, fir.rs:15); with
 * decim D > 1 only outputs at stream indices D-1, 2D-1, ... are produced (the reference
 * computes all and Decimate drops D-1 of every D; only the kept ones are computed here).
 * State (ntaps-1 history, decimation phase) carries across process() calls, so any
 * partition of a stream into blocks gives the same outputs.  An inf / NaN sample makes
 * exactly the outputs non-finite whose ntaps-sample window holds it, as in the reference
 * (every algorithm recomputes such outputs with the reference's sequential sum).
 * Kinds: (F32,F32), (C64,F32), (C64,C64), and (CU8,F32), (CU8,C64) for rtl_tcp u8 IQ
 * (the reference's rtl.listen().filter(...) chain, examples/live.rs:29-31, src/main.rs:38-49):
 * the (v-128)/128 conversion is fused into the FIR load (decim 4 with f32 taps runs on the
 * MFMA path at 2 input bytes per sample); history and outputs are C64.
 * (F32 samples with C64 taps do not type-check in the reference: f32 is not
 * Mul<Complex<f32>, Output=f32>.)
 * ===================================================================================== */
typedef struct sdrgpu_fir sdrgpu_fir;

int sdrgpu_fir_create(int device, int sample_kind, int tap_kind, const void* taps,
                      size_t ntaps, uint32_t decim, sdrgpu_fir** out);
int sdrgpu_fir_set_algorithm(sdrgpu_fir* h, int algo);
/* Use an external hipStream_t (NULL restores the handle's own stream). */
int sdrgpu_fir_set_stream(sdrgpu_fir* h, void* hip_stream);
int sdrgpu_fir_get_stream(const sdrgpu_fir* h, void** hip_stream);
/* Number of outputs the next process() call produces for n_in inputs. */
int sdrgpu_fir_output_len(const sdrgpu_fir* h, size_t n_in, size_t* n_out);
int sdrgpu_fir_process(sdrgpu_fir* h, const void* in, size_t n_in, void* out,
                       size_t out_cap, size_t* n_out);
/* DEVICE pointers, enqueued on the handle's stream.  d_out may overlap d_in (in place, or
 * shifted): the handle then filters a device copy of the input, so the results are those of an
 * out-of-place call (the kernels store output tiles while other workgroups still read the
 * input under them).  The same holds for sdrgpu_firbank_process_dev, sdrgpu_fft_exec_dev,
 * sdrgpu_rfft_exec_dev and sdrgpu_stft_process_dev. */
int sdrgpu_fir_process_dev(sdrgpu_fir* h, const void* d_in, size_t n_in, void* d_out,
                           size_t out_cap, size_t* n_out);
/* HOST pointers, asynchronous (the Block adapter's producer/consumer split,
 * src/signal/adapters/block.rs:105-207): H2D + FIR + D2H are enqueued on the handle's
 * stream and the call returns with *n_out set.  Use pinned buffers (sdrgpu_host_alloc) --
 * pageable ones work but the copies then block -- keep `in` unchanged and read `out` only
 * after sdrgpu_fir_sync.  Double-buffering two blocks keeps PCIe busy in both directions
 * of the pipeline while the host prepares the next block. */
int sdrgpu_fir_process_async(sdrgpu_fir* h, const void* in, size_t n_in, void* out,
                             size_t out_cap, size_t* n_out);
int sdrgpu_fir_sync(sdrgpu_fir* h);
/* The algorithm (SDRGPU_FIR_DIRECT / _OVERLAP_SAVE / _MATRIX) that ran the most recent
 * non-empty block; SDRGPU_FIR_AUTO before the first one.  Introspection for tests and
 * benches (which kernel family a shape actually took); no reference counterpart. */
int sdrgpu_fir_last_algorithm(const sdrgpu_fir* h, int* algo);
int sdrgpu_fir_last_kernel(const sdrgpu_fir* h, int* kernel);  /* sdrgpu_fir_kernel */
int sdrgpu_fir_reset(sdrgpu_fir* h);                           /* FilterDesign::design -> fresh state */
int sdrgpu_fir_clone(const sdrgpu_fir* h, sdrgpu_fir** out);   /* #[derive(Clone)] Fir, fir.rs:6 */
void sdrgpu_fir_destroy(sdrgpu_fir* h);

/* Batched FIR bank: nch independent channels sharing one tap set, per-channel state.
 * Channel c's samples start at in + c*ld_in (ld in samples).  Same semantics per
 * channel as sdrgpu_fir (each channel is one Fir, src/filter/fir.rs:6-32). */
typedef struct sdrgpu_firbank sdrgpu_firbank;

int sdrgpu_firbank_create(int device, int sample_kind, int tap_kind, const void* taps,
                          size_t ntaps, uint32_t decim, size_t nch, sdrgpu_firbank** out);
int sdrgpu_firbank_set_algorithm(sdrgpu_firbank* h, int algo);
int sdrgpu_firbank_set_stream(sdrgpu_firbank* h, void* hip_stream);
int sdrgpu_firbank_get_stream(const sdrgpu_firbank* h, void** hip_stream);
int sdrgpu_firbank_output_len(const sdrgpu_firbank* h, size_t n_in, size_t* n_out);
int sdrgpu_firbank_process(sdrgpu_firbank* h, const void* in, size_t ld_in, size_t n_in,
                           void* out, size_t ld_out, size_t* n_out);
int sdrgpu_firbank_process_dev(sdrgpu_firbank* h, const void* d_in, size_t ld_in,
                               size_t n_in, void* d_out, size_t ld_out, size_t* n_out);
int sdrgpu_firbank_sync(sdrgpu_firbank* h);
int sdrgpu_firbank_last_algorithm(const sdrgpu_firbank* h, int* algo);
int sdrgpu_firbank_last_kernel(const sdrgpu_firbank* h, int* kernel);
int sdrgpu_firbank_reset(sdrgpu_firbank* h);
int sdrgpu_firbank_clone(const sdrgpu_firbank* h, sdrgpu_firbank** out);
void sdrgpu_firbank_destroy(sdrgpu_firbank* h);

/* =====================================================================================
 * FFT.
 * Replaces: fft::fft  (src/fft.rs:3-28)  -- forward DFT, fftshift collate, x 1/sqrt(N)
 *           fft::rfft (src/fft.rs:30-37)  -- real input, keeps output bins [N/2, N)
 * exec transforms `count` back-to-back frames of n C64 samples; out[i] of each frame is
 * X[(i - n/2) mod n] / sqrt(n) (fft.rs:14-26).  Frequencies (fft.rs:18,24) are
 * (i - n/2) * rate / n and are produced host-side by sdrgpu_fft_freqs.
 * Any n >= 1 plans, as rustfft's FFTplanner does (fft.rs:10-11): powers of two up to 2^20
 * run the Stockham / four-step kernels; other n whose prime factors are all <= 13 run
 * mixed-radix tiles (n <= 4096) or a mixed-radix four-step (n = n1*n2, both <= 4096); the
 * rest run Bluestein over a power-of-two convolution (n <= 2^19).  Larger n:
 * SDRGPU_ERR_UNSUPPORTED.
 * ===================================================================================== */
typedef struct sdrgpu_fft sdrgpu_fft;

int sdrgpu_fft_plan(int device, size_t n, sdrgpu_fft** out);
int sdrgpu_fft_set_stream(sdrgpu_fft* h, void* hip_stream);
int sdrgpu_fft_get_stream(const sdrgpu_fft* h, void** hip_stream);
int sdrgpu_fft_exec(sdrgpu_fft* h, const void* in, void* out, size_t count);
int sdrgpu_fft_exec_dev(sdrgpu_fft* h, const void* d_in, void* d_out, size_t count);
/* rfft: `count` frames of n F32 samples -> count frames of n - n/2 C64 values: the collated
 * output with its first n/2 entries drained (fft.rs:35), i.e. X[0 .. n - n/2) * 1/sqrt(n). */
int sdrgpu_rfft_exec(sdrgpu_fft* h, const float* in, void* out, size_t count);
/* rfft on device pointers (count frames of n F32 in, n - n/2 outputs each out), enqueued
 * on the plan's stream. */
int sdrgpu_rfft_exec_dev(sdrgpu_fft* h, const float* d_in, void* d_out, size_t count);
/* Output format of exec / rfft_exec (and the STFT): SDRGPU_FFT_OUT_COMPLEX (default, C64) or
 * SDRGPU_FFT_OUT_DB -- one f32 per bin, 20*log10(|X * 1/sqrt(n)|): the magnitude-in-dB
 * conversion every spectrum plot of the reference applies to fft's output
 * (ComplexSeries with db = true: y.norm(), then 20 * log10, src/plot/complexseries.rs:90-92;
 * examples/fft.rs:80-100, examples/live.rs), fused into the transform's store (half the
 * output bytes). */
enum sdrgpu_fft_output { SDRGPU_FFT_OUT_COMPLEX = 0, SDRGPU_FFT_OUT_DB = 1 };
int sdrgpu_fft_set_output(sdrgpu_fft* h, int mode);
int sdrgpu_fft_sync(sdrgpu_fft* h);
void sdrgpu_fft_destroy(sdrgpu_fft* h);
int sdrgpu_fft_freqs(size_t n, float rate, float* freqs);

/* STFT = sig.window(n/rate).decimate(rate/hop).map(fft::fft)  (examples/live.rs:29-39):
 * Window keeps the last n samples zero-prefilled (src/signal/adapters/mod.rs:277-299);
 * Decimate(wait=hop) yields a frame after every hop-th input (adapters/mod.rs:30-37).
 * Frame j covers stream samples [(j+1)hop - n, (j+1)hop).  Streaming: state carries
 * across calls. */
typedef struct sdrgpu_stft sdrgpu_stft;

int sdrgpu_stft_create(int device, size_t n, size_t hop, sdrgpu_stft** out);
int sdrgpu_stft_set_stream(sdrgpu_stft* h, void* hip_stream);
int sdrgpu_stft_get_stream(const sdrgpu_stft* h, void** hip_stream);
int sdrgpu_stft_output_len(const sdrgpu_stft* h, size_t n_in, size_t* n_frames);
int sdrgpu_stft_process(sdrgpu_stft* h, const void* in, size_t n_in, void* out,
                        size_t out_cap_frames, size_t* n_frames);
int sdrgpu_stft_process_dev(sdrgpu_stft* h, const void* d_in, size_t n_in, void* d_out,
                            size_t out_cap_frames, size_t* n_frames);
/* HOST pointers, asynchronous (as sdrgpu_fir_process_async): H2D + frames enqueued on the
 * handle's stream, the download on a second stream; pinned buffers (sdrgpu_host_alloc), `in`
 * unchanged and `out` unread until sdrgpu_stft_sync. */
int sdrgpu_stft_process_async(sdrgpu_stft* h, const void* in, size_t n_in, void* out,
                              size_t out_cap_frames, size_t* n_frames);
/* SDRGPU_C64 (default) or SDRGPU_CU8: raw rtl_tcp I/Q bytes as examples/live.rs feeds
 * rtl.listen() into window(..) (src/rtltcp.rs:156-164 conversion done in the frame load). */
int sdrgpu_stft_set_input_kind(sdrgpu_stft* h, int sample_kind);
int sdrgpu_stft_set_output(sdrgpu_stft* h, int mode);  /* sdrgpu_fft_output */
int sdrgpu_stft_sync(sdrgpu_stft* h);
int sdrgpu_stft_reset(sdrgpu_stft* h);
void sdrgpu_stft_destroy(sdrgpu_stft* h);

/* =====================================================================================
 * Biquad designs and batched PLL.
 * Replaces: BiquadD::design (src/filter/biquad.rs:73-155), Biquad::new/apply (:25-56),
 *           filter::Identity (src/filter/simple.rs:3-19),
 *           PllDesign::new/design (src/filter/pll.rs:25-60), Pll::apply (:70-85).
 * One PLL per channel; output[i] = Some(output) -> value, None -> 0.0 (src/main.rs:49
 * unwrap_or(0.0)), locked[i] = 1 when Some.
 * ===================================================================================== */
enum sdrgpu_biquad_kind {
    SDRGPU_BQ_IDENTITY = 0,
    SDRGPU_BQ_LOWPASS = 1,   /* BiquadD::LowPass(freq, q)  */
    SDRGPU_BQ_HIGHPASS = 2,  /* BiquadD::HighPass(freq, q) */
    SDRGPU_BQ_BANDPASS = 3,  /* BiquadD::BandPass(freq, q) */
    SDRGPU_BQ_NOTCH = 4,     /* BiquadD::Notch(freq, q)    */
    SDRGPU_BQ_LR = 5,        /* BiquadD::Lr(decayrate) -- freq field, q ignored */
};
typedef struct { int32_t kind; float freq; float q; } sdrgpu_biquad_design;

typedef struct {
    float reference;                 /* PllDesign::new reference (Hz)  */
    float gain;                      /* PllDesign::new gain            */
    float rate;                      /* FilterDesign::design(rate)     */
    sdrgpu_biquad_design loopf;      /* on Complex<f32>                */
    sdrgpu_biquad_design outputf;    /* on f32                         */
    sdrgpu_biquad_design lockf;      /* on f32                         */
} sdrgpu_pll_params;

typedef struct sdrgpu_pll sdrgpu_pll;

int sdrgpu_pll_create(int device, const sdrgpu_pll_params* p, size_t nch, sdrgpu_pll** out);
/* What `out` receives (the lock mask is unchanged):
 *   SDRGPU_PLL_OUT_FILTER (default): output filter of phasedif * rate, 0.0 when unlocked
 *     (Pll::apply, pll.rs:79-84; None -> 0.0 as src/main.rs:49);
 *   SDRGPU_PLL_OUT_STEREO_DIFF: the FM stereo pilot map of src/main.rs:58-66 -- the input is
 *     Complex::new(v, 0.0) and out = (v / value.powi(2)).re * 0.5 with the PLL's updated NCO
 *     value when locked, else 0.0 (mono = v * 0.5 stays on the caller). */
enum sdrgpu_pll_output { SDRGPU_PLL_OUT_FILTER = 0, SDRGPU_PLL_OUT_STEREO_DIFF = 1 };
int sdrgpu_pll_set_output_mode(sdrgpu_pll* h, int mode);
/* Input samples: SDRGPU_C64 (default) or SDRGPU_CU8 -- raw rtl_tcp I/Q byte pairs
 * (src/main.rs:48-49 feeds rtl.listen() straight into the PLL), converted in the load as
 * RtlTcpSignal::next does, (v - 128) / 128 (src/rtltcp.rs:156-164); ld_in counts samples. */
int sdrgpu_pll_set_input_kind(sdrgpu_pll* h, int sample_kind);
/* Time-parallel blocks (no reference counterpart; results are the serial PLL's bit for bit):
 * each channel's block is cut into segments of `seg` samples that run concurrently, each after
 * `warm` samples of warm-up from the design state; segments whose warm-up did not reach the
 * true state exactly are re-run in parallel from their predecessor's end state and, where that
 * was not true either, recomputed from the true state.  seg = 0: automatic
 * (enough segments to give every SIMD one wave, none shorter than 4096 samples), seg < 0:
 * always one serial pass; warm = 0: 4096.  Lengths round up to multiples of 8.  The automatic
 * plan adapts per handle: after a block in which more than half of the segments had to be
 * recomputed (an unlocked loop, e.g. noise with no station), the next 8 blocks run one serial
 * pass and the handle then tries segments again (reset starts over).  A
 * sdrgpu_pll_process_dev call whose output or lock range overlaps its input range (in place)
 * runs one serial pass whatever the plan (the segment kernels re-read inputs after outputs are
 * stored). */
int sdrgpu_pll_set_time_parallel(sdrgpu_pll* h, long seg, long warm);
/* The segment length (0 = one serial pass) and warm-up a block of n samples would use. */
int sdrgpu_pll_time_parallel_plan(const sdrgpu_pll* h, size_t n, long* seg, long* warm);
/* The most recent block: its segment count (0 = serial) and how many segments had to be
 * recomputed from the true state (waits for the handle's stream). */
int sdrgpu_pll_last_time_parallel(sdrgpu_pll* h, long* segments, long* recomputed);
/* Measurement aid (no reference counterpart): with on != 0, time-parallel blocks record HIP
 * events around their three kernels -- pass 1 (segments with warm-up), the parallel re-run pass
 * and the per-channel walk -- and sdrgpu_pll_last_phase_ms returns the most recent block's
 * three times in ms (all 0 for a serial block or with timing off; waits for the stream). */
int sdrgpu_pll_set_phase_timing(sdrgpu_pll* h, int on);
int sdrgpu_pll_last_phase_ms(sdrgpu_pll* h, float* pass1, float* rerun, float* walk);
int sdrgpu_pll_set_stream(sdrgpu_pll* h, void* hip_stream);
int sdrgpu_pll_get_stream(const sdrgpu_pll* h, void** hip_stream);
int sdrgpu_pll_process(sdrgpu_pll* h, const void* in, size_t ld_in, size_t n,
                       float* out, uint8_t* locked, size_t ld_out);
int sdrgpu_pll_process_dev(sdrgpu_pll* h, const void* d_in, size_t ld_in, size_t n,
                           float* d_out, uint8_t* d_locked, size_t ld_out);
/* HOST pointers, asynchronous: nch x n dense blocks (ld = n) in, out / locked dense; H2D +
 * PLL on the handle's stream, downloads on a second stream (the Block hand-off in front of
 * the PLL, src/main.rs:47-49).  Pinned buffers; read outputs after sdrgpu_pll_sync. */
int sdrgpu_pll_process_async(sdrgpu_pll* h, const void* in, size_t n, float* out,
                             uint8_t* locked);
/* Public Pll fields nphase / value (src/filter/pll.rs:20-21) of channel ch. */
int sdrgpu_pll_state(sdrgpu_pll* h, size_t ch, float* nphase, float* value_re_im);
int sdrgpu_pll_sync(sdrgpu_pll* h);
int sdrgpu_pll_reset(sdrgpu_pll* h);
int sdrgpu_pll_clone(const sdrgpu_pll* h, sdrgpu_pll** out);
void sdrgpu_pll_destroy(sdrgpu_pll* h);

/* Diagnostics (test-only, no reference counterpart): evaluates on `device` the libm
 * restatements the PLL kernels inline for Pll::apply's arg() and from_polar (pll.rs:72-76;
 * num-complex calls f32::atan2 / sin / cos, i.e. glibc atan2f / sinf / cosf on x86-64 Linux),
 * so their special-operand paths can be compared bit for bit with glibc.  HOST pointers,
 * synchronous.  SDRGPU_DEBUG_ATAN2F: out0[i] = atan2f(a[i], b[i]) (y = a, x = b);
 * SDRGPU_DEBUG_SINCOSF: out0[i] = sinf(a[i]), out1[i] = cosf(a[i]) (b unused), valid for
 * |a| < 120 (the PLL's phase argument is 2*pi*nphase, |nphase| < 1). */
enum sdrgpu_debug_fn { SDRGPU_DEBUG_ATAN2F = 0, SDRGPU_DEBUG_SINCOSF = 1 };
int sdrgpu_debug_libm(int device, int fn, const float* a, const float* b, float* out0,
                      float* out1, size_t n);

/* Batched biquad: nch independent Biquad<C, f32> filters (C = F32 or C64) designed by
 * BiquadD::design(rate) (src/filter/biquad.rs:73-155; SDRGPU_BQ_IDENTITY = filter::Identity,
 * src/filter/simple.rs:3-19), applied as Signal::filter (src/signal/mod.rs:42-48) with
 * Biquad::apply's DF1 recurrence in the reference's f32 operation order (biquad.rs:42-56):
 * outputs are bit-identical to the reference.  Channel c at in + c*ld_in samples.  The
 * de-emphasis stage of the FM receiver (BiquadD::Lr, src/main.rs:52,75-81) is one of these. */
typedef struct sdrgpu_biquad sdrgpu_biquad;

int sdrgpu_biquad_create(int device, int sample_kind, const sdrgpu_biquad_design* d, float rate,
                         size_t nch, sdrgpu_biquad** out);
/* b0 b1 b2 na1 na2 as Biquad::new normalises them (biquad.rs:25-38) */
int sdrgpu_biquad_coefs(const sdrgpu_biquad* h, float* coefs5);
int sdrgpu_biquad_set_stream(sdrgpu_biquad* h, void* hip_stream);
int sdrgpu_biquad_get_stream(const sdrgpu_biquad* h, void** hip_stream);
int sdrgpu_biquad_process(sdrgpu_biquad* h, const void* in, size_t ld_in, size_t n, void* out,
                          size_t ld_out);
int sdrgpu_biquad_process_dev(sdrgpu_biquad* h, const void* d_in, size_t ld_in, size_t n,
                              void* d_out, size_t ld_out);
/* Time-parallel blocks (no reference counterpart: Biquad::apply is serial, biquad.rs:42-56;
 * outputs stay identical to it).  A channel's block is cut into segments of `seg` samples
 * that run at once, each after `warm` samples of warm-up from zero output history, verified
 * bit for bit against the true state and recomputed where they differ.  seg = warm = 0:
 * automatic (warm-up from the filter's slower pole, enough segments to fill the device, none
 * for Identity, an unstable design or a block that gives fewer than two); seg < 0: always
 * one serial pass.  Mirrors sdrgpu_pll_set_time_parallel, in-place calls included (an output
 * range overlapping the input runs one serial pass). */
int sdrgpu_biquad_set_time_parallel(sdrgpu_biquad* h, long seg, long warm);
/* the (segment, warm-up) a block of n samples per channel would use (segment 0: serial) */
int sdrgpu_biquad_time_parallel_plan(const sdrgpu_biquad* h, size_t n, long* seg, long* warm);
/* segments per channel of the most recent block (0: serial) and how many missed their guess
 * (synchronizes the handle's stream) */
int sdrgpu_biquad_last_time_parallel(sdrgpu_biquad* h, long* segments, long* recomputed);
int sdrgpu_biquad_sync(sdrgpu_biquad* h);
int sdrgpu_biquad_reset(sdrgpu_biquad* h);
int sdrgpu_biquad_clone(const sdrgpu_biquad* h, sdrgpu_biquad** out);
void sdrgpu_biquad_destroy(sdrgpu_biquad* h);

/* =====================================================================================
 * Sample-rate conversion: the libsamplerate surface src/resample.rs binds through
 * libsamplerate-sys (SampleRate::new -> src_new :32-44, process -> src_process :46-67,
 * reset -> src_reset :72-77, try_clone -> src_clone :79-86, channels -> src_get_channels
 * :88-92, set_ratio -> src_set_ratio :94-99, Drop -> src_delete :103-110, version
 * :3-8, ConverterType::name/description :121-135, Error::description :189-196), so the
 * Rust wrapper swaps `src_*` for `sdrgpu_src_*` and keeps its Error::from_c mapping
 * (:236-262): these functions return LIBSAMPLERATE error codes (0 = ok, 1..22 as in
 * sdrgpu_src_error below), not sdrgpu_status.
 *
 * Converters: SDRGPU_SRC_ZERO_ORDER_HOLD and SDRGPU_SRC_LINEAR follow libsamplerate's
 * src_zoh.c / src_linear.c exactly (f64 position walk, f32 samples, state carried across
 * calls).  The three sinc converters follow libsamplerate 0.2's src_sinc.c (buffer
 * handling, fixed-point filter index, ratio ramp, end-of-input flush, f64 sums) with our own
 * Kaiser-windowed sinc tables of libsamplerate's increments and lengths -- its coefficient
 * headers are not in this image, so their outputs are not libsamplerate's.
 * end_of_input is honoured as there (the Rust wrapper sets it for an empty input slice,
 * whose pointer is non-NULL: pass a non-NULL data_in to flush).
 *
 * Frames hold `channels` interleaved f32 (f32 = 1, Complex<f32> = 2, (A, B) = sum;
 * src/resample.rs:272-282); a large channel count batches many independent streams that
 * share one ratio.  sdrgpu_src_process takes HOST pointers and is synchronous;
 * sdrgpu_src_process_dev takes DEVICE pointers, fills the frame counts at once and
 * enqueues the conversion on the handle's stream (sdrgpu_src_sync to wait).
 * ===================================================================================== */
enum sdrgpu_src_converter {       /* libsamplerate's converter ids */
    SDRGPU_SRC_SINC_BEST_QUALITY = 0,
    SDRGPU_SRC_SINC_MEDIUM_QUALITY = 1,
    SDRGPU_SRC_SINC_FASTEST = 2,
    SDRGPU_SRC_ZERO_ORDER_HOLD = 3,
    SDRGPU_SRC_LINEAR = 4,
};
enum sdrgpu_src_error {           /* libsamplerate's codes, as src/resample.rs:208-234 */
    SDRGPU_SRC_ERR_MALLOC_FAILED = 1,
    SDRGPU_SRC_ERR_BAD_STATE = 2,
    SDRGPU_SRC_ERR_BAD_DATA = 3,
    SDRGPU_SRC_ERR_BAD_DATA_PTR = 4,
    SDRGPU_SRC_ERR_BAD_SRC_RATIO = 6,
    SDRGPU_SRC_ERR_BAD_CONVERTER = 10,
    SDRGPU_SRC_ERR_BAD_CHANNEL_COUNT = 11,
    SDRGPU_SRC_ERR_DATA_OVERLAP = 16,
    SDRGPU_SRC_ERR_SINC_PREPARE_DATA_BAD_LEN = 21,
    SDRGPU_SRC_ERR_BAD_INTERNAL_STATE = 22,
};
/* layout of libsamplerate's SRC_DATA (the struct SampleRate::process fills, :47-56) */
typedef struct {
    const float* data_in;
    float* data_out;
    long input_frames, output_frames;
    long input_frames_used, output_frames_gen;
    int end_of_input;
    double src_ratio;             /* output rate / input rate, in [1/256, 256] */
} sdrgpu_src_data;

typedef struct sdrgpu_src_state sdrgpu_src_state;
sdrgpu_src_state* sdrgpu_src_new(int device, int converter_type, int channels, int* error);
int sdrgpu_src_process(sdrgpu_src_state* s, sdrgpu_src_data* data);
int sdrgpu_src_process_dev(sdrgpu_src_state* s, sdrgpu_src_data* data);
int sdrgpu_src_sync(sdrgpu_src_state* s);
int sdrgpu_src_reset(sdrgpu_src_state* s);
sdrgpu_src_state* sdrgpu_src_clone(sdrgpu_src_state* s, int* error);
int sdrgpu_src_get_channels(sdrgpu_src_state* s);   /* negative error code on a null handle */
int sdrgpu_src_set_ratio(sdrgpu_src_state* s, double new_ratio);
int sdrgpu_src_set_stream(sdrgpu_src_state* s, void* hip_stream);
int sdrgpu_src_get_stream(sdrgpu_src_state* s, void** hip_stream);
sdrgpu_src_state* sdrgpu_src_delete(sdrgpu_src_state* s);  /* returns NULL, as src_delete */
const char* sdrgpu_src_strerror(int error);
const char* sdrgpu_src_get_name(int converter_type);        /* NULL for unknown ids */
const char* sdrgpu_src_get_description(int converter_type);
const char* sdrgpu_src_get_version(void);
/* The coefficient table of sinc converter 0..2 (length returned; coeffs == NULL asks for
 * the length only; *increment = the table's index increment).  -1 for other ids or a
 * short buffer.  Not in libsamplerate's API: the tables are this library's own. */
int sdrgpu_src_sinc_table(int converter_type, float* coeffs, int cap, int* increment);

/* =====================================================================================
 * Multi-GPU channel sharding (configs[4]: channels sharded across the GPUs of one node).
 * No reference counterpart (the reference is single-process CPU code):
 * channels are independent, so the only collectives are the fan-out of channel blocks from
 * a root and the gather of results back -- RCCL over xGMI, one process per GPU.  The
 * 128-byte unique id is created on rank 0 and shared out of band (e.g. torch.distributed
 * over gloo).  Byte counts are per rank; buffers are device pointers.
 * ===================================================================================== */
typedef struct sdrgpu_comm sdrgpu_comm;
#define SDRGPU_COMM_ID_BYTES 128

int sdrgpu_comm_unique_id(void* id_out /* SDRGPU_COMM_ID_BYTES */);
int sdrgpu_comm_init(int device, int nranks, int rank, const void* id, sdrgpu_comm** out);
/* root's d_send holds nranks consecutive blocks of bytes_per_rank; rank i gets block i */
int sdrgpu_comm_scatter(sdrgpu_comm* c, const void* d_send, void* d_recv, size_t bytes_per_rank,
                        int root, void* hip_stream);
/* rank i's block lands at d_recv + i*bytes_per_rank on root */
int sdrgpu_comm_gather(sdrgpu_comm* c, const void* d_send, void* d_recv, size_t bytes_per_rank,
                       int root, void* hip_stream);
/* Uneven channel blocks (nch % nranks != 0): bytes[r] / displs[r] (nranks host entries,
 * the same on every rank) give rank r's block size and its offset in the root's buffer.
 * Grouped point-to-point sends from / receives to the root (ncclSend / ncclRecv). */
int sdrgpu_comm_scatterv(sdrgpu_comm* c, const void* d_send, const size_t* bytes,
                         const size_t* displs, void* d_recv, int root, void* hip_stream);
int sdrgpu_comm_gatherv(sdrgpu_comm* c, const void* d_send, void* d_recv, const size_t* bytes,
                        const size_t* displs, int root, void* hip_stream);
int sdrgpu_comm_barrier(sdrgpu_comm* c, void* hip_stream);
void sdrgpu_comm_destroy(sdrgpu_comm* c);

/* The point-to-point plan scatterv (gather = 0) / gatherv (gather = 1) issue on `rank`:
 * one op per non-empty transfer -- a zero-byte rank (nch < nranks) takes part in no send,
 * receive or copy.  kind: SDRGPU_COMM_SEND / RECV (peer = the other rank) or
 * SDRGPU_COMM_COPY (the root's own block, a device-local copy; peer = root); offset = the
 * byte offset of the block in the ROOT's buffer (displs[r]; 0 on the non-root side, whose
 * buffer holds only its own block).  Host-only arithmetic, no device work: *n_ops = the op
 * count (ops may be NULL to ask for it; SDRGPU_ERR_INVALID if max_ops is short). */
typedef struct {
    int32_t kind;
    int32_t peer;
    size_t offset;
    size_t bytes;
} sdrgpu_comm_op;
enum { SDRGPU_COMM_SEND = 0, SDRGPU_COMM_RECV = 1, SDRGPU_COMM_COPY = 2 };
int sdrgpu_comm_plan_v(int nranks, int rank, int root, int gather, const size_t* bytes,
                       const size_t* displs, sdrgpu_comm_op* ops, int max_ops, int* n_ops);

#ifdef __cplusplus
}
#endif
#endif /* SDRGPU_H */
