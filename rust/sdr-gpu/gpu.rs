//! `src/gpu.rs` for the `sdr` crate (agrif/unnamed-rust-sdr): safe drop-ins over
//! libsdrgpu.so (raw bindings: rust/sdrgpu-sys, generated from include/sdrgpu.h).
//!
//! To use: copy this file to the crate's `src/gpu.rs`, add `pub mod gpu;` to `src/lib.rs`
//! and `sdrgpu-sys = { path = "<repo>/rust/sdrgpu-sys" }` to `[dependencies]`
//!.  It follows the crate's only existing FFI wrapper, `src/resample.rs`
//! over libsamplerate-sys: an opaque `*mut` handle, status codes mapped to an `Error`
//! (`src/resample.rs:151-270`), `Clone` through a native clone call, `Drop` through
//! destroy, `unsafe impl Send` and no `Sync` (`src/resample.rs:23-25`; the `Block` adapter
//! moves filters across rayon workers, `src/signal/adapters/block.rs:142-146`).
//!
//! Not compiled in this repository's image (no Rust toolchain); the same ABI is driven by
//! the Python mirror and the GPU test suite, and tests/test_rust_binding.py checks every
//! `sys::` call below against include/sdrgpu.h (name and argument count).
//!
//! Drop-in map (reference -> here):
//!   `signal.filter(taps)` (Fir, src/filter/fir.rs:6-58)      -> `signal.filter(GpuFirD::new(taps))`
//!   `.filter(taps).decimate(r)` (adapters/mod.rs:13-41)      -> `.filter_block(GpuFirBlock::new(..))`
//!   `PllDesign::new(..)` (src/filter/pll.rs:25-60)           -> `GpuPllDesign::new(..)` (same args)
//!   `BiquadD` as a stage (src/filter/biquad.rs:73-155)       -> `GpuBiquadD(BiquadD::..)`
//!   `fft::fft` / `fft::rfft` (src/fft.rs:3-37)               -> `gpu::fft` / `gpu::rfft`
//!   `window(..).decimate(..).map(fft)` (examples/live.rs)   -> `GpuStft::new(sig, n, hop)`
//!   `SampleRate` (src/resample.rs)                           -> same code, `sdrgpu_src_*` symbols

use std::collections::VecDeque;
use std::ptr;

use num::Complex;
use sdrgpu_sys as sys;

use crate::filter::{BiquadD, Filter, FilterDesign, Identity};
use crate::Signal;

// ------------------------------------------------------------------------------- errors

/// A non-zero sdrgpu status (include/sdrgpu.h `enum sdrgpu_status`), in the style of
/// `resample::Error` (src/resample.rs:151-270).
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct Error(pub i32);

impl std::fmt::Display for Error {
    fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
        let msg = unsafe { std::ffi::CStr::from_ptr(sys::sdrgpu_strerror(self.0)) };
        write!(f, "sdrgpu error {}: {}", self.0, msg.to_string_lossy())
    }
}

impl std::error::Error for Error {}

pub type Result<T> = std::result::Result<T, Error>;

fn check(code: i32) -> Result<()> {
    if code == sys::SDRGPU_OK {
        Ok(())
    } else {
        Err(Error(code))
    }
}

/// GPU the handles below are created on (one process per GPU: set by the launcher).
pub const DEVICE: i32 = 0;

// ------------------------------------------------------------------------------ samples

/// Sample layouts the ABI accepts, like `resample::Resample`'s layout contract
/// (src/resample.rs:28-30, 272-282): `f32` and `num::Complex<f32>` (`#[repr(C)]` re/im).
pub unsafe trait GpuSample: Copy + num::Zero {
    const KIND: i32;
}
unsafe impl GpuSample for f32 {
    const KIND: i32 = sys::SDRGPU_F32;
}
unsafe impl GpuSample for Complex<f32> {
    const KIND: i32 = sys::SDRGPU_C64;
}

// ------------------------------------------------------------------------- FIR, D = 1

/// Drop-in for `Fir<C, A>` (src/filter/fir.rs:6-32): `Filter<A>` with `Output = A`, zero
/// initial history (fir.rs:15), state carried from call to call.  `apply` is one FFI call
/// per sample (API parity only); pipelines pass blocks through `process` or the
/// `GpuFilterBlock` adapter below.
pub struct GpuFir<A> {
    h: *mut sys::sdrgpu_fir,
    out: Vec<A>,
}

unsafe impl<A> Send for GpuFir<A> {}

impl<A: GpuSample> GpuFir<A> {
    pub fn new<C: GpuSample>(coef: &[C]) -> Result<Self> {
        let mut h = ptr::null_mut();
        check(unsafe {
            sys::sdrgpu_fir_create(DEVICE, A::KIND, C::KIND, coef.as_ptr() as *const _,
                                   coef.len(), 1, &mut h)
        })?;
        Ok(GpuFir { h, out: Vec::new() })
    }

    /// One block: `output` gets exactly `input.len()` samples (D = 1), as if `apply` had
    /// been called on each (`SampleRate::process`'s shape, src/resample.rs:46-67).
    pub fn process(&mut self, input: &[A], output: &mut Vec<A>) -> Result<usize> {
        output.resize(input.len(), A::zero());
        let mut n = 0;
        check(unsafe {
            sys::sdrgpu_fir_process(self.h, input.as_ptr() as *const _, input.len(),
                                    output.as_mut_ptr() as *mut _, output.len(), &mut n)
        })?;
        output.truncate(n);
        Ok(n)
    }

    /// `FilterDesign::design` again: a fresh history (fir.rs:12-19).
    pub fn reset(&mut self) -> Result<()> {
        check(unsafe { sys::sdrgpu_fir_reset(self.h) })
    }
}

impl<A: GpuSample> Filter<A> for GpuFir<A> {
    type Output = A;
    fn apply(&mut self, value: A) -> A {
        let mut out = std::mem::take(&mut self.out);
        self.process(&[value], &mut out).expect("sdrgpu_fir_process");
        let y = out[0];
        self.out = out;
        y
    }
}

impl<A> Clone for GpuFir<A> {
    // #[derive(Clone)] on Fir (fir.rs:6): the copy carries the history
    fn clone(&self) -> Self {
        let mut h = ptr::null_mut();
        check(unsafe { sys::sdrgpu_fir_clone(self.h, &mut h) }).expect("sdrgpu_fir_clone");
        GpuFir { h, out: Vec::new() }
    }
}

impl<A> Drop for GpuFir<A> {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_fir_destroy(self.h) }
    }
}

/// `FilterDesign` for taps (fir.rs:36-58): `signal.filter(GpuFirD::new(taps))` replaces
/// `signal.filter(taps)` with the same `Output = A`.
#[derive(Clone, Debug)]
pub struct GpuFirD<C> {
    pub coef: Vec<C>,
}

impl<C> GpuFirD<C> {
    pub fn new(coef: Vec<C>) -> Self {
        GpuFirD { coef }
    }
}

impl<A: GpuSample, C: GpuSample> FilterDesign<A> for GpuFirD<C> {
    type Output = A;
    type Filter = GpuFir<A>;
    fn design(self, _rate: f32) -> GpuFir<A> {
        GpuFir::new(&self.coef).expect("sdrgpu_fir_create")
    }
}

// ------------------------------------------------------------- FIR + fused decimation

/// `Fir` followed by `Decimate(D)` (adapters/mod.rs:13-41) with only the kept outputs
/// (stream indices D-1, 2D-1, ...) computed.  Per-sample `Filter` output is `Option<A>`:
/// `None` for the D-1 samples `Decimate` drops.  Also takes rtl_tcp bytes (`new_cu8`:
/// `(v - 128) / 128`, src/rtltcp.rs:156-164, folded into the FIR load).
pub struct GpuFirDecim<A> {
    h: *mut sys::sdrgpu_fir,
    decim: u32,
    out: Vec<A>,
}

unsafe impl<A> Send for GpuFirDecim<A> {}

impl<A: GpuSample> GpuFirDecim<A> {
    pub fn new<C: GpuSample>(coef: &[C], decim: u32) -> Result<Self> {
        Self::with_kind(A::KIND, coef, decim)
    }

    fn with_kind<C: GpuSample>(kind: i32, coef: &[C], decim: u32) -> Result<Self> {
        let mut h = ptr::null_mut();
        check(unsafe {
            sys::sdrgpu_fir_create(DEVICE, kind, C::KIND, coef.as_ptr() as *const _, coef.len(),
                                   decim, &mut h)
        })?;
        Ok(GpuFirDecim { h, decim, out: Vec::new() })
    }

    fn run(&mut self, input: *const u8, n_in: usize, output: &mut Vec<A>) -> Result<usize> {
        let mut n = 0;
        check(unsafe { sys::sdrgpu_fir_output_len(self.h, n_in, &mut n) })?;
        output.resize(n, A::zero());
        check(unsafe {
            sys::sdrgpu_fir_process(self.h, input as *const _, n_in,
                                    output.as_mut_ptr() as *mut _, n, &mut n)
        })?;
        output.truncate(n);
        Ok(n)
    }

    pub fn process(&mut self, input: &[A], output: &mut Vec<A>) -> Result<usize> {
        self.run(input.as_ptr() as *const u8, input.len(), output)
    }

    pub fn decim(&self) -> u32 {
        self.decim
    }
}

impl GpuFirDecim<Complex<f32>> {
    /// rtl_tcp I/Q bytes as read from the socket (RtlTcpConnection::read,
    /// src/rtltcp.rs:136-140), 2 bytes per sample, converted inside the FIR load.
    pub fn new_cu8(coef: &[f32], decim: u32) -> Result<Self> {
        Self::with_kind(sys::SDRGPU_CU8, coef, decim)
    }

    pub fn process_cu8(&mut self, iq: &[u8], output: &mut Vec<Complex<f32>>) -> Result<usize> {
        self.run(iq.as_ptr(), iq.len() / 2, output)
    }
}

impl<A: GpuSample> Filter<A> for GpuFirDecim<A> {
    type Output = Option<A>;
    fn apply(&mut self, value: A) -> Option<A> {
        let mut out = std::mem::take(&mut self.out);
        self.process(&[value], &mut out).expect("sdrgpu_fir_process");
        let y = out.pop();
        self.out = out;
        y
    }
}

impl<A> Drop for GpuFirDecim<A> {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_fir_destroy(self.h) }
    }
}

// ----------------------------------------------------------------------- FIR bank

/// `nch` independent `Fir`s sharing one tap set (one `Fir` per channel, fir.rs:6-32):
/// the matched filter of configs[3] and the channelizer of configs[4].  Channel c's
/// samples are `input[c * ld .. c * ld + n]`.
pub struct GpuFirBank<A> {
    h: *mut sys::sdrgpu_firbank,
    nch: usize,
    _a: std::marker::PhantomData<A>,
}

unsafe impl<A> Send for GpuFirBank<A> {}

impl<A: GpuSample> GpuFirBank<A> {
    pub fn new<C: GpuSample>(coef: &[C], decim: u32, nch: usize) -> Result<Self> {
        let mut h = ptr::null_mut();
        check(unsafe {
            sys::sdrgpu_firbank_create(DEVICE, A::KIND, C::KIND, coef.as_ptr() as *const _,
                                       coef.len(), decim, nch, &mut h)
        })?;
        Ok(GpuFirBank { h, nch, _a: std::marker::PhantomData })
    }

    /// `input`: nch rows of `n` samples (leading dimension n); returns outputs per channel.
    pub fn process(&mut self, input: &[A], n: usize, output: &mut Vec<A>) -> Result<usize> {
        assert_eq!(input.len(), self.nch * n);
        let mut m = 0;
        check(unsafe { sys::sdrgpu_firbank_output_len(self.h, n, &mut m) })?;
        output.resize(self.nch * m.max(1), A::zero());
        check(unsafe {
            sys::sdrgpu_firbank_process(self.h, input.as_ptr() as *const _, n, n,
                                        output.as_mut_ptr() as *mut _, m.max(1), &mut m)
        })?;
        output.truncate(self.nch * m);
        Ok(m)
    }

    pub fn reset(&mut self) -> Result<()> {
        check(unsafe { sys::sdrgpu_firbank_reset(self.h) })
    }
}

impl<A> Drop for GpuFirBank<A> {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_firbank_destroy(self.h) }
    }
}

// ------------------------------------------------------------------ biquad designs

/// The filter designs the PLL and the biquad stage take: `BiquadD` (src/filter/biquad.rs:
/// 73-155) and `Identity` (src/filter/simple.rs:3-19).  The coefficients are designed on
/// the host in f32 exactly as `BiquadD::design` does (include/sdrgpu.h).
pub trait GpuBiquadDesign {
    fn to_sys(&self) -> sys::sdrgpu_biquad_design;
}

impl GpuBiquadDesign for BiquadD {
    fn to_sys(&self) -> sys::sdrgpu_biquad_design {
        let (kind, freq, q) = match *self {
            BiquadD::LowPass(f, q) => (sys::SDRGPU_BQ_LOWPASS, f, q),
            BiquadD::HighPass(f, q) => (sys::SDRGPU_BQ_HIGHPASS, f, q),
            BiquadD::BandPass(f, q) => (sys::SDRGPU_BQ_BANDPASS, f, q),
            BiquadD::Notch(f, q) => (sys::SDRGPU_BQ_NOTCH, f, q),
            BiquadD::Lr(decay) => (sys::SDRGPU_BQ_LR, decay, 0.0),
        };
        sys::sdrgpu_biquad_design { kind, freq, q }
    }
}

impl GpuBiquadDesign for Identity {
    fn to_sys(&self) -> sys::sdrgpu_biquad_design {
        sys::sdrgpu_biquad_design { kind: sys::SDRGPU_BQ_IDENTITY, freq: 0.0, q: 0.0 }
    }
}

/// `nch` independent `Biquad<f32, A>` (DF1, the reference's f32 operation order, outputs
/// bit-identical): e.g. the de-emphasis `Lr` stage of src/main.rs:52,75-81.
pub struct GpuBiquad<A> {
    h: *mut sys::sdrgpu_biquad,
    nch: usize,
    _a: std::marker::PhantomData<A>,
}

unsafe impl<A> Send for GpuBiquad<A> {}

impl<A: GpuSample> GpuBiquad<A> {
    pub fn new<D: GpuBiquadDesign>(design: &D, rate: f32, nch: usize) -> Result<Self> {
        let d = design.to_sys();
        let mut h = ptr::null_mut();
        check(unsafe { sys::sdrgpu_biquad_create(DEVICE, A::KIND, &d, rate, nch, &mut h) })?;
        Ok(GpuBiquad { h, nch, _a: std::marker::PhantomData })
    }

    pub fn process(&mut self, input: &[A], n: usize, output: &mut Vec<A>) -> Result<()> {
        assert_eq!(input.len(), self.nch * n);
        output.resize(self.nch * n, A::zero());
        check(unsafe {
            sys::sdrgpu_biquad_process(self.h, input.as_ptr() as *const _, n, n,
                                       output.as_mut_ptr() as *mut _, n)
        })
    }

    /// Long blocks of few channels run as verified speculative segments by default (outputs
    /// identical to Biquad::apply's serial recurrence); `seg < 0` forces one serial pass,
    /// `(0, 0)` restores the automatic plan.
    pub fn set_time_parallel(&mut self, seg: i64, warm: i64) -> Result<()> {
        check(unsafe { sys::sdrgpu_biquad_set_time_parallel(self.h, seg as _, warm as _) })
    }
}

impl<A: GpuSample> Filter<A> for GpuBiquad<A> {
    type Output = A;
    fn apply(&mut self, value: A) -> A {
        let mut out = Vec::with_capacity(1);
        self.process(&[value], 1, &mut out).expect("sdrgpu_biquad_process");
        out[0]
    }
}

impl<A> Drop for GpuBiquad<A> {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_biquad_destroy(self.h) }
    }
}

/// `signal.filter(GpuBiquadD(BiquadD::Lr(..)))` for `signal.filter(BiquadD::Lr(..))`.
#[derive(Clone, Copy, Debug)]
pub struct GpuBiquadD(pub BiquadD);

impl<A: GpuSample> FilterDesign<A> for GpuBiquadD {
    type Output = A;
    type Filter = GpuBiquad<A>;
    fn design(self, rate: f32) -> GpuBiquad<A> {
        GpuBiquad::new(&self.0, rate, 1).expect("sdrgpu_biquad_create")
    }
}

// ------------------------------------------------------------------------------- PLL

/// `PllDesign::new(reference, gain, loopfilter, outputfilter, lockfilter)` with the same
/// arguments (src/filter/pll.rs:25-37); `design(rate)` gives a `GpuPll` whose outputs and
/// lock decisions are bit-identical to `Pll::apply` (pll.rs:70-85).
#[derive(Clone, Debug)]
pub struct GpuPllDesign<Loop, Output, Lock> {
    reference: f32,
    gain: f32,
    loopfilter: Loop,
    outputfilter: Output,
    lockfilter: Lock,
}

impl<Loop, Output, Lock> GpuPllDesign<Loop, Output, Lock>
where
    Loop: GpuBiquadDesign,
    Output: GpuBiquadDesign,
    Lock: GpuBiquadDesign,
{
    pub fn new(reference: f32, gain: f32, loopfilter: Loop, outputfilter: Output,
               lockfilter: Lock) -> Self {
        GpuPllDesign { reference, gain, loopfilter, outputfilter, lockfilter }
    }

    /// `nch` independent loops in one handle (the batched form of configs[3]).
    pub fn design_batch(&self, rate: f32, nch: usize) -> Result<GpuPll> {
        let p = sys::sdrgpu_pll_params {
            reference: self.reference,
            gain: self.gain,
            rate,
            loopf: self.loopfilter.to_sys(),
            outputf: self.outputfilter.to_sys(),
            lockf: self.lockfilter.to_sys(),
        };
        let mut h = ptr::null_mut();
        check(unsafe { sys::sdrgpu_pll_create(DEVICE, &p, nch, &mut h) })?;
        Ok(GpuPll { h, nch, v: Vec::new(), l: Vec::new() })
    }
}

impl<Loop, Output, Lock> FilterDesign<Complex<f32>> for GpuPllDesign<Loop, Output, Lock>
where
    Loop: GpuBiquadDesign,
    Output: GpuBiquadDesign,
    Lock: GpuBiquadDesign,
{
    type Output = Option<f32>;
    type Filter = GpuPll;
    fn design(self, rate: f32) -> GpuPll {
        self.design_batch(rate, 1).expect("sdrgpu_pll_create")
    }
}

pub struct GpuPll {
    h: *mut sys::sdrgpu_pll,
    nch: usize,
    v: Vec<f32>,
    l: Vec<u8>,
}

unsafe impl Send for GpuPll {}

impl GpuPll {
    /// `input`: nch rows of n samples.  `Some(v)` / `None` per sample as Pll::apply's lock
    /// test decides (pll.rs:80-84).
    pub fn process(&mut self, input: &[Complex<f32>], n: usize,
                   out: &mut Vec<Option<f32>>) -> Result<()> {
        assert_eq!(input.len(), self.nch * n);
        self.v.resize(self.nch * n, 0.0);
        self.l.resize(self.nch * n, 0);
        check(unsafe {
            sys::sdrgpu_pll_process(self.h, input.as_ptr() as *const _, n, n,
                                    self.v.as_mut_ptr(), self.l.as_mut_ptr(), n)
        })?;
        out.clear();
        out.extend(self.v.iter().zip(&self.l).map(|(v, l)| if *l != 0 { Some(*v) } else { None }));
        Ok(())
    }

    /// src/main.rs:48-49: rtl.listen() bytes straight into the loop ((v - 128) / 128 in the load)
    pub fn set_input_cu8(&mut self) -> Result<()> {
        check(unsafe { sys::sdrgpu_pll_set_input_kind(self.h, sys::SDRGPU_CU8) })
    }

    /// src/main.rs:54-69: output (v / value.powi(2)).re * 0.5 while locked (stereo pilot)
    pub fn set_stereo_diff_output(&mut self) -> Result<()> {
        check(unsafe { sys::sdrgpu_pll_set_output_mode(self.h, sys::SDRGPU_PLL_OUT_STEREO_DIFF) })
    }

    /// The public fields `nphase`, `value` of channel `ch` (pll.rs:20-21).
    pub fn state(&self, ch: usize) -> Result<(f32, Complex<f32>)> {
        let (mut nphase, mut v) = (0f32, [0f32; 2]);
        check(unsafe { sys::sdrgpu_pll_state(self.h, ch, &mut nphase, v.as_mut_ptr()) })?;
        Ok((nphase, Complex::new(v[0], v[1])))
    }

    pub fn reset(&mut self) -> Result<()> {
        check(unsafe { sys::sdrgpu_pll_reset(self.h) })
    }

    /// Long blocks run as verified speculative segments by default (outputs identical to
    /// Pll::apply's serial recurrence); `seg < 0` forces one serial pass, `(0, 0)` restores
    /// the automatic plan.
    pub fn set_time_parallel(&mut self, seg: i64, warm: i64) -> Result<()> {
        check(unsafe { sys::sdrgpu_pll_set_time_parallel(self.h, seg as _, warm as _) })
    }
}

impl Filter<Complex<f32>> for GpuPll {
    type Output = Option<f32>;
    fn apply(&mut self, value: Complex<f32>) -> Option<f32> {
        let mut o = Vec::with_capacity(1);
        self.process(&[value], 1, &mut o).expect("sdrgpu_pll_process");
        o[0]
    }
}

impl Clone for GpuPll {
    // #[derive(Clone)] on Pll (pll.rs:12)
    fn clone(&self) -> Self {
        let mut h = ptr::null_mut();
        check(unsafe { sys::sdrgpu_pll_clone(self.h, &mut h) }).expect("sdrgpu_pll_clone");
        GpuPll { h, nch: self.nch, v: Vec::new(), l: Vec::new() }
    }
}

impl Drop for GpuPll {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_pll_destroy(self.h) }
    }
}

// ------------------------------------------------------------------------------- FFT

fn freqs(n: usize, rate: f32) -> Vec<f32> {
    let mut f = vec![0f32; n];
    check(unsafe { sys::sdrgpu_fft_freqs(n, rate, f.as_mut_ptr()) }).expect("sdrgpu_fft_freqs");
    f
}

/// A planned n-point transform (plan once, unlike fft.rs:10-11 which plans per call).
pub struct GpuFftPlan {
    h: *mut sys::sdrgpu_fft,
    n: usize,
}

unsafe impl Send for GpuFftPlan {}

impl GpuFftPlan {
    pub fn new(n: usize) -> Result<Self> {
        let mut h = ptr::null_mut();
        check(unsafe { sys::sdrgpu_fft_plan(DEVICE, n, &mut h) })?;
        Ok(GpuFftPlan { h, n })
    }

    /// `count` frames of n samples -> collated, 1/sqrt(n)-normalised spectra (fft.rs:14-26).
    pub fn exec(&mut self, input: &[Complex<f32>], output: &mut Vec<Complex<f32>>) -> Result<()> {
        let count = input.len() / self.n;
        output.resize(count * self.n, Complex::new(0.0, 0.0));
        check(unsafe {
            sys::sdrgpu_fft_exec(self.h, input.as_ptr() as *const _,
                                 output.as_mut_ptr() as *mut _, count)
        })
    }

    /// rfft frames (fft.rs:30-37): n - n/2 values per frame.
    pub fn exec_real(&mut self, input: &[f32], output: &mut Vec<Complex<f32>>) -> Result<()> {
        let count = input.len() / self.n;
        output.resize(count * (self.n - self.n / 2), Complex::new(0.0, 0.0));
        check(unsafe {
            sys::sdrgpu_rfft_exec(self.h, input.as_ptr(), output.as_mut_ptr() as *mut _, count)
        })
    }
}

impl Drop for GpuFftPlan {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_fft_destroy(self.h) }
    }
}

/// `fft::fft` (src/fft.rs:3-28): same signature and output, any length.
pub fn fft<S: Signal<Sample = Complex<f32>>>(input: S) -> Vec<(f32, Complex<f32>)> {
    let rate = input.rate();
    let data: Vec<Complex<f32>> = input.iter().collect();
    let n = data.len();
    if n == 0 {
        return Vec::new();
    }
    let mut out = Vec::new();
    GpuFftPlan::new(n).and_then(|mut p| p.exec(&data, &mut out)).expect("sdrgpu fft");
    freqs(n, rate).into_iter().zip(out).collect()
}

/// `fft::rfft` (src/fft.rs:30-37): the collated output with its first n/2 entries drained.
pub fn rfft<S: Signal<Sample = f32>>(input: S) -> Vec<(f32, Complex<f32>)> {
    let rate = input.rate();
    let data: Vec<f32> = input.iter().collect();
    let n = data.len();
    if n == 0 {
        return Vec::new();
    }
    let mut out = Vec::new();
    GpuFftPlan::new(n).and_then(|mut p| p.exec_real(&data, &mut out)).expect("sdrgpu rfft");
    let mut f = freqs(n, rate);
    f.drain(..n / 2);
    f.into_iter().zip(out).collect()
}

// ------------------------------------------------------------------------ Signal adapters

/// `signal.filter(taps).decimate(rate)` as one Signal stage, modelled on
/// `adapters::Resample` (src/signal/adapters/resample.rs:38-82): refill a block from
/// upstream, run it through the GPU, hand samples out one at a time.  `rate()` keeps the
/// `Decimate::rate` quirk (the upstream rate, adapters/mod.rs:38-40).
pub struct GpuFilterBlock<S: Signal> {
    signal: S,
    fir: GpuFirDecim<S::Sample>,
    inbuf: Vec<S::Sample>,
    outbuf: Vec<S::Sample>,
    pos: usize,
    block: usize,
}

impl<S: Signal> GpuFilterBlock<S>
where
    S::Sample: GpuSample,
{
    /// `block` = seconds of input per GPU call (like `Signal::block(size)`, block.rs:117)
    pub fn new<C: GpuSample>(signal: S, coef: &[C], decim: u32, block: f32) -> Result<Self> {
        let n = ((block * signal.rate()).ceil() as usize).max(decim as usize);
        Ok(GpuFilterBlock {
            fir: GpuFirDecim::new(coef, decim)?,
            signal,
            inbuf: Vec::with_capacity(n),
            outbuf: Vec::new(),
            pos: 0,
            block: n,
        })
    }
}

impl<S: Signal> Signal for GpuFilterBlock<S>
where
    S::Sample: GpuSample,
{
    type Sample = S::Sample;
    fn next(&mut self) -> Option<S::Sample> {
        while self.pos >= self.outbuf.len() {
            self.inbuf.clear();
            while self.inbuf.len() < self.block {
                match self.signal.next() {
                    Some(v) => self.inbuf.push(v),
                    None => break,
                }
            }
            if self.inbuf.is_empty() {
                return None;
            }
            self.fir.process(&self.inbuf, &mut self.outbuf).expect("sdrgpu_fir_process");
            self.pos = 0;
        }
        self.pos += 1;
        Some(self.outbuf[self.pos - 1])
    }
    fn rate(&self) -> f32 {
        self.signal.rate()
    }
}

/// `sig.window(n / rate).decimate(rate / hop).map(|w| fft::fft(..))` (examples/live.rs:29-39)
/// as one Signal: each `next()` is one frame's `Vec<(f32, Complex<f32>)>`.
pub struct GpuStft<S: Signal> {
    signal: S,
    h: *mut sys::sdrgpu_stft,
    n: usize,
    block: Vec<Complex<f32>>,
    frames: VecDeque<Vec<(f32, Complex<f32>)>>,
    freqs: Vec<f32>,
    buf: Vec<Complex<f32>>,
}

impl<S: Signal<Sample = Complex<f32>>> GpuStft<S> {
    pub fn new(signal: S, n: usize, hop: usize) -> Result<Self> {
        let mut h = ptr::null_mut();
        check(unsafe { sys::sdrgpu_stft_create(DEVICE, n, hop, &mut h) })?;
        let freqs = freqs(n, signal.rate());
        Ok(GpuStft { signal, h, n, block: Vec::with_capacity(8 * hop), frames: VecDeque::new(),
                     freqs, buf: Vec::new() })
    }
}

impl<S: Signal<Sample = Complex<f32>>> Signal for GpuStft<S> {
    type Sample = Vec<(f32, Complex<f32>)>;
    fn next(&mut self) -> Option<Self::Sample> {
        while self.frames.is_empty() {
            self.block.clear();
            while self.block.len() < self.block.capacity() {
                match self.signal.next() {
                    Some(v) => self.block.push(v),
                    None => break,
                }
            }
            if self.block.is_empty() {
                return None;
            }
            let mut nf = 0;
            check(unsafe { sys::sdrgpu_stft_output_len(self.h, self.block.len(), &mut nf) })
                .expect("sdrgpu_stft_output_len");
            self.buf.resize(nf.max(1) * self.n, Complex::new(0.0, 0.0));
            check(unsafe {
                sys::sdrgpu_stft_process(self.h, self.block.as_ptr() as *const _, self.block.len(),
                                         self.buf.as_mut_ptr() as *mut _, nf.max(1), &mut nf)
            })
            .expect("sdrgpu_stft_process");
            for f in 0..nf {
                let fr = &self.buf[f * self.n..(f + 1) * self.n];
                self.frames.push_back(self.freqs.iter().cloned().zip(fr.iter().cloned()).collect());
            }
        }
        self.frames.pop_front()
    }
    fn rate(&self) -> f32 {
        self.signal.rate() // Decimate::rate quirk (adapters/mod.rs:38-40)
    }
}

impl<S: Signal> Drop for GpuStft<S> {
    fn drop(&mut self) {
        unsafe { sys::sdrgpu_stft_destroy(self.h) }
    }
}

// ----------------------------------------------------------- async pinned block streaming

/// Pinned host memory (sdrgpu_host_alloc): copies from / to it are DMA and do not block.
pub struct PinnedBuf {
    p: *mut u8,
    bytes: usize,
}

unsafe impl Send for PinnedBuf {}

impl PinnedBuf {
    pub fn new(bytes: usize) -> Result<Self> {
        let mut p = ptr::null_mut();
        check(unsafe { sys::sdrgpu_host_alloc(DEVICE, bytes, &mut p) })?;
        Ok(PinnedBuf { p: p as *mut u8, bytes })
    }
    pub fn as_mut_slice<T: Copy>(&mut self) -> &mut [T] {
        unsafe { std::slice::from_raw_parts_mut(self.p as *mut T, self.bytes / std::mem::size_of::<T>()) }
    }
}

impl Drop for PinnedBuf {
    fn drop(&mut self) {
        unsafe {
            sys::sdrgpu_host_free(self.p as *mut _);
        }
    }
}

/// `Block` (src/signal/adapters/block.rs:105-207) with the GPU as the consumer: the producer
/// fills one pinned slot while the other is uploaded, filtered and downloaded
/// (sdrgpu_fir_process_async: H2D + FIR on the handle's stream, D2H on a second one).
pub struct GpuBlockFir {
    fir: GpuFirDecim<Complex<f32>>,
    inb: [PinnedBuf; 2],
    outb: [PinnedBuf; 2],
    n_out: [usize; 2],
    slot: usize,
    block: usize,
}

impl GpuBlockFir {
    pub fn new(coef: &[f32], decim: u32, block: usize) -> Result<Self> {
        let ib = block * std::mem::size_of::<Complex<f32>>();
        let ob = (block / decim as usize + 1) * std::mem::size_of::<Complex<f32>>();
        Ok(GpuBlockFir {
            fir: GpuFirDecim::new(coef, decim)?,
            inb: [PinnedBuf::new(ib)?, PinnedBuf::new(ib)?],
            outb: [PinnedBuf::new(ob)?, PinnedBuf::new(ob)?],
            n_out: [0, 0],
            slot: 0,
            block,
        })
    }

    /// the slot the producer fills next
    pub fn input(&mut self) -> &mut [Complex<f32>] {
        let s = self.slot;
        self.inb[s].as_mut_slice()
    }

    /// hand the filled slot (first `n_in` samples) to the GPU and return at once
    pub fn submit(&mut self, n_in: usize) -> Result<()> {
        assert!(n_in <= self.block);
        let s = self.slot;
        let cap = self.outb[s].bytes / std::mem::size_of::<Complex<f32>>();
        check(unsafe {
            sys::sdrgpu_fir_process_async(self.fir.h, self.inb[s].p as *const _, n_in,
                                          self.outb[s].p as *mut _, cap, &mut self.n_out[s])
        })?;
        self.slot ^= 1;
        Ok(())
    }

    /// wait for everything submitted; slot `s`'s outputs are then `output(s)`
    pub fn wait(&mut self) -> Result<()> {
        check(unsafe { sys::sdrgpu_fir_sync(self.fir.h) })
    }

    pub fn output(&mut self, s: usize) -> &[Complex<f32>] {
        let n = self.n_out[s];
        &self.outb[s].as_mut_slice::<Complex<f32>>()[..n]
    }
}
