// pll.hip -- batched PLL / FM demodulator (one channel per lane) for gfx950.
//
// Semantics: Pll::apply (reference src/filter/pll.rs:70-85) with BiquadD loop / output /
// lock filters (src/filter/biquad.rs:25-56, 83-155) or Identity (src/filter/simple.rs:3-19):
//   c = x * conj(v);  phasedif = arg(loop(c)) * gain;  nphase = fract(nphase + ref + phasedif)
//   v = from_polar(1, 2 pi nphase);  locked = lock(c.re);  out = output(phasedif * rate)
//   -> Some(out) if locked > 0.01 else None   (None written as 0.0, src/main.rs:49)
// out_mode 1 writes the stereo difference signal of src/main.rs:58-66 instead of `out`.
//
// The recurrence is serial and nonlinear (atan2 -> NCO -> sin/cos each sample), so it is
// latency-bound, not HBM- or FLOP-bound: a channel costs the issue of its
// per-sample instruction stream (one wave per SIMD at 1024 channels), so every instruction
// off the recurrence counts; the next 8 samples of every lane are in flight while the
// current 8 are processed.
//
// Bit-exact by construction: on noisy input the reference loop is chaotic (a 1-ulp change
// in one sample moves the next cycle slip; FMA vs no-FMA builds of the same code differ by
// 3 % L2), so this kernel reproduces the reference arithmetic exactly: this file is built
// with -ffp-contract=off, every operation is written in the reference's order (num-complex
// Mul, Biquad::apply's `0 + v*b0 + x1*b1 + ...`), and sin/cos/atan2 are the bit-exact
// restatements of the glibc functions Rust std calls (libm_glibc.h).
#include <algorithm>
#include <cstddef>
#include <type_traits>

#include "common.hpp"
#include "libm_glibc.h"
#include "pll_kernels.hpp"

namespace sdrgpu {

namespace {

constexpr int kPllBlock = 64;   // one wave: 64 channels
constexpr int kChunk = 8;       // samples per lane per pipeline stage

// Every PLL wave owns its SIMD: the kernels claim the whole register file (v255 and a255 are
// named, so each wave allocates 512 VGPRs and no other wave -- of any kernel -- can be resident
// on that SIMD while it runs).  Measured reason (round 5, DESIGN 3.6, profiles/r05_chain_probe.txt):
// with two waves of a D = 1 MFMA FIR bank on the same SIMD (a bank build at 201 VGPRs leaves
// room for a 96-VGPR PLL wave), the chain wave's mixer c = x * conj(v) -- a v_pk_mul_f32 whose
// result the next v_pk_add_f32 reads -- came out as c.re = x.re * v.re in lanes 48-63 at one
// sample (the product y * v.im read as 0), and the chaotic loop then diverged; inputs, the
// NCO value and the LDS hand-off were all right, and nothing in the ISA orders one wave's
// VALU results against another wave's.  With the SIMD to itself the chain is bit-exact again,
// at the same speed (a PLL wave alone on its SIMD is what it is sized for anyway).
__device__ __forceinline__ void own_simd() { claim_simd_whole(); }

struct Bq {
    float b0, b1, b2, na1, na2;
};

// Biquad::apply on f32 (biquad.rs:43-56), reference order, no contraction.
__device__ __forceinline__ float bq_real(const Bq& c, float x, float& x1, float& x2, float& y1,
                                         float& y2) {
    float out = 0.0f;
    out += x * c.b0;
    out += x1 * c.b1;
    out += x2 * c.b2;
    out += y1 * c.na1;
    out += y2 * c.na2;
    x2 = x1;
    x1 = x;
    y2 = y1;
    y1 = out;
    return out;
}

// U8: samples are rtl_tcp byte pairs, converted as RtlTcpSignal::next does
// ((v as f32 - 128.0) / 128.0, src/rtltcp.rs:156-164 -- exact in f32) inside the load.
// LID / OID / KID: loop / output / lock filter is Identity (1), a biquad (0) or read from the
// parameters at run time (2); MODE: output mode 0 / 1, or 2 = run time.  The designs of the
// reference's callers are compiled as their own kernels (src/main.rs:41-46: loop LowPass,
// output Identity, lock LowPass; examples/pll.rs:9-15: three LowPass; the stereo pilot
// src/main.rs:55-60), so no per-sample control flow is left in them.
template <int LID, int OID, int KID, int MODE>
struct PllLane {
    Bq L, O, K;
    float gain, reference, rate;
    bool loop_id, out_id, lock_id;
    int mode;
    __device__ explicit PllLane(const PllDevParams& p)
        : L{p.loopc[0], p.loopc[1], p.loopc[2], p.loopc[3], p.loopc[4]},
          O{p.outc[0], p.outc[1], p.outc[2], p.outc[3], p.outc[4]},
          K{p.lockc[0], p.lockc[1], p.lockc[2], p.lockc[3], p.lockc[4]},
          gain(p.gain), reference(p.reference), rate(p.rate),
          loop_id(LID == 2 ? p.loop_ident != 0 : LID == 1),
          out_id(OID == 2 ? p.out_ident != 0 : OID == 1),
          lock_id(KID == 2 ? p.lock_ident != 0 : KID == 1),
          mode(MODE == 2 ? p.out_mode : MODE) {}

    // one reference Pll::apply step; returns (output or 0, locked)
    __device__ __forceinline__ void step(PllChannelState& s, float2 v, float& ov, uint8_t& lv) const {
        constexpr float kTwoPi = 2.0f * 3.14159265358979323846f;  // 2.0 * f32::consts::PI
        // c = value * conj(self.value)  (pll.rs:71; num-complex 0.2 Mul)
        const float cjr = s.vr, cji = -s.vi;
        const float cr = v.x * cjr - v.y * cji;
        const float ci = v.x * cji + v.y * cjr;
        float lr = cr, li = ci;
        if (!loop_id) {
            // Biquad<f32, Complex<f32>>::apply: Convolve::accumulate = out += a * c
            float orr = 0.0f, oi = 0.0f;
            orr += cr * L.b0;      oi += ci * L.b0;
            orr += s.lx1r * L.b1;  oi += s.lx1i * L.b1;
            orr += s.lx2r * L.b2;  oi += s.lx2i * L.b2;
            orr += s.ly1r * L.na1; oi += s.ly1i * L.na1;
            orr += s.ly2r * L.na2; oi += s.ly2i * L.na2;
            s.lx2r = s.lx1r; s.lx1r = cr; s.ly2r = s.ly1r; s.ly1r = orr;
            s.lx2i = s.lx1i; s.lx1i = ci; s.ly2i = s.ly1i; s.ly1i = oi;
            lr = orr;
            li = oi;
        }
        const float phasedif = sdr_atan2f_bfx(li, lr) * gain;     // :72 arg() * gain
        float nph = s.nphase + (reference + phasedif);             // :73
        nph = nph - truncf(nph);                                   // :74 fract()
        s.nphase = nph;
        const float phase = kTwoPi * nph;                          // :75
        float sn, cs;
        sdr_sincosf_bf2(phase, &sn, &cs);                          // glibc sinf/cosf, branch-free
        s.vr = 1.0f * cs;                                          // :76 from_polar
        s.vi = 1.0f * sn;
        // off the loop-carried chain: lock / output filters and the output select
        const float lockv = lock_id ? cr : bq_real(K, cr, s.kx1, s.kx2, s.ky1, s.ky2);  // :78
        const float o = out_id ? phasedif * rate
                               : bq_real(O, phasedif * rate, s.ox1, s.ox2, s.oy1, s.oy2);
        const bool lockd = lockv > 0.01f;                          // :80
        lv = lockd ? 1 : 0;
        if (mode == 1) {
            // src/main.rs:58-66, the stereo pilot: input = Complex::new(v, 0.0);
            // diff = (v / value.powi(2)).re * 0.5 when locked.  powi(2) = value * value
            // (num-complex Mul); f32 / Complex: re = v * w.re / norm_sqr(w)
            const float wr = s.vr * s.vr - s.vi * s.vi;
            const float wi = s.vr * s.vi + s.vi * s.vr;
            const float nrm = wr * wr + wi * wi;
            const float dre = v.x * wr / nrm;
            ov = lockd ? dre * 0.5f : 0.0f;
        } else {
            ov = lockd ? o : 0.0f;
        }
    }
};

__device__ __forceinline__ float2 cvt_u8(unsigned w) {
    return make_float2(((float)(w & 255u) - 128.0f) / 128.0f, ((float)((w >> 8) & 255u) - 128.0f) / 128.0f);
}

// Samples [a, b) of one channel row through the step.  STORE: outputs and lock flags to y / lk
// (indexed like the input); otherwise only the state advances (a warm-up).  VEC: the row is
// 16-B aligned (ld_in even, or a multiple of 8 for u8 input), a is a multiple of kChunk and
// y / lk are 16-B / 8-B aligned at a multiple of kChunk, so a chunk of 8 samples moves in 4
// (c64) or 1 (u8) loads and 3 stores, the next chunk's loads in flight.
template <bool U8, bool VEC, bool STORE, class Lane>
__device__ __forceinline__ void pll_run(const Lane& ln, PllChannelState& s, const void* __restrict__ row,
                                        long a, long b, float* __restrict__ y,
                                        uint8_t* __restrict__ lk) {
    const float2* __restrict__ xf = static_cast<const float2*>(row);
    const unsigned short* __restrict__ xu = static_cast<const unsigned short*>(row);
    auto ld = [&](long i) -> float2 {
        if constexpr (U8) return cvt_u8(xu[i]);
        else return xf[i];
    };
    using RawT = std::conditional_t<U8, uint4, float4>;
    constexpr int NR = U8 ? 1 : kChunk / 2;  // raw vector loads per chunk
    const long bfull = a + (b - a) / kChunk * kChunk;
    RawT raw[NR];
    auto ldc = [&](long i) {  // chunk starting at sample i
        if constexpr (VEC) {
            const RawT* q = reinterpret_cast<const RawT*>(U8 ? (const void*)(xu + i) : (const void*)(xf + i));
#pragma unroll
            for (int r = 0; r < NR; ++r) raw[r] = q[r];
        }
    };
    auto sample = [&](int k, long i) -> float2 {
        if constexpr (VEC) {
            if constexpr (U8) {
                const unsigned w = (&raw[0].x)[k >> 1];
                return cvt_u8((k & 1) ? (w >> 16) : (w & 0xffffu));
            } else {
                const float4 r = raw[k >> 1];
                return (k & 1) ? make_float2(r.z, r.w) : make_float2(r.x, r.y);
            }
        } else {
            return ld(i + k);
        }
    };
    float2 buf[kChunk];
    if (bfull > a) {
        ldc(a);
#pragma unroll
        for (int k = 0; k < kChunk; ++k) buf[k] = sample(k, a);
    }
    for (long i = a; i < bfull; i += kChunk) {
        float2 cur[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) cur[k] = buf[k];
        if (i + kChunk < bfull) {  // prefetch
            ldc(i + kChunk);
#pragma unroll
            for (int k = 0; k < kChunk; ++k) buf[k] = sample(k, i + kChunk);
        }
        float ov[kChunk];
        uint8_t lv[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) ln.step(s, cur[k], ov[k], lv[k]);
        if constexpr (STORE) {
            if constexpr (VEC) {
                float4* yo = reinterpret_cast<float4*>(y + i);
                yo[0] = make_float4(ov[0], ov[1], ov[2], ov[3]);
                yo[1] = make_float4(ov[4], ov[5], ov[6], ov[7]);
                uint2 pk;
                pk.x = lv[0] | (lv[1] << 8) | (lv[2] << 16) | ((unsigned)lv[3] << 24);
                pk.y = lv[4] | (lv[5] << 8) | (lv[6] << 16) | ((unsigned)lv[7] << 24);
                *reinterpret_cast<uint2*>(lk + i) = pk;
            } else {
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    y[i + k] = ov[k];
                    lk[i + k] = lv[k];
                }
            }
        }
    }
    // ragged tail: exactly b - bfull more samples (the state must not see padding)
    for (long i = bfull; i < b; ++i) {
        float o;
        uint8_t l;
        ln.step(s, ld(i), o, l);
        if constexpr (STORE) {
            y[i] = o;
            lk[i] = l;
        }
    }
}

template <bool U8, int LID, int OID, int KID, int MODE, bool VEC>
__global__ __launch_bounds__(kPllBlock) void pll_kernel(PllDevParams p, const void* __restrict__ in_,
                                                        long ld_in, long n, float* __restrict__ out,
                                                        uint8_t* __restrict__ locked, long ld_out,
                                                        PllChannelState* __restrict__ state) {
    own_simd();
    const long ch = (long)blockIdx.x * kPllBlock + threadIdx.x;
    if (ch >= p.nch) return;
    PllChannelState s = state[ch];
    const PllLane<LID, OID, KID, MODE> ln(p);
    const void* row = static_cast<const char*>(in_) + ch * ld_in * (U8 ? 2 : 8);
    pll_run<U8, VEC, true>(ln, s, row, 0, n, out + ch * ld_out, locked + ch * ld_out);
    state[ch] = s;
}

// Time-parallel PLL ("speculative segments").  The recurrence is serial, but a PLL that is
// tracking forgets its initial state: from any start, the whole state (NCO phase and value,
// loop / lock / output filter states) comes to agree BIT FOR BIT with the true trajectory after
// a few thousand samples of the same input (configs[3]'s FM channels: median 3.4 k, max 12 k
// samples in 128 channels).  So each channel's block is cut into segments that
// run at once, one lane each (pll_seg_kernel): a segment first runs `warm` samples of warm-up
// from the design state (no outputs), records the state it reached at its start (guess), then
// produces its outputs and records its end state.  pll_fix_kernel (one lane per channel) then
// walks the segments in order with the TRUE state (segment 0 starts from the carried state;
// so does every segment whose warm-up reaches back to sample 0): where a segment's guess equals
// the true state bit for bit, its outputs are exactly the serial ones (same state, same inputs,
// same arithmetic) and its end state is true; where it differs, the segment is recomputed from
// the true state.  Every output is therefore the serial PLL's; only the time depends on how
// many segments have to be recomputed (none, typically; all of them for a chaotic, unlocked
// loop, which then costs one serial pass more than pll_kernel).
template <bool U8, int LID, int OID, int KID, int MODE, bool VEC>
__global__ __launch_bounds__(kPllBlock) void pll_seg_kernel(
    PllDevParams p, const void* __restrict__ in_, long ld_in, long n, float* __restrict__ out,
    uint8_t* __restrict__ locked, long ld_out, const PllChannelState* __restrict__ state, long seg,
    long warm, long nseg, PllChannelState* __restrict__ guess, PllChannelState* __restrict__ endst,
    long ck, PllChannelState* __restrict__ ckpt) {
    own_simd();
    const long g = (long)blockIdx.x * kPllBlock + threadIdx.x;
    if (g >= p.nch * nseg) return;
    const long ch = g % p.nch, sg = g / p.nch;
    const long t0 = sg * seg, t1 = t0 + seg < n ? t0 + seg : n, tw = t0 > warm ? t0 - warm : 0;
    PllChannelState s{};  // PllDesign::design's state (pll.rs:57-58) unless the warm-up starts at 0
    if (tw == 0) s = state[ch];
    const PllLane<LID, OID, KID, MODE> ln(p);
    const void* row = static_cast<const char*>(in_) + ch * ld_in * (U8 ? 2 : 8);
    pll_run<U8, VEC, false>(ln, s, row, tw, t0, nullptr, nullptr);
    guess[g] = s;
    // the segment in checkpoint intervals: a recomputation from the true state can stop where
    // it meets this trajectory (pll_fix_kernel)
    const long nck = seg / ck;
    PllChannelState* __restrict__ cp = ckpt + g * (nck - 1);
    for (long j = 0; j < nck; ++j) {
        const long a = t0 + j * ck, b = j + 1 < nck ? (a + ck < t1 ? a + ck : t1) : t1;
        if (a >= b) break;
        pll_run<U8, VEC, true>(ln, s, row, a, b, out + ch * ld_out, locked + ch * ld_out);
        if (j + 1 < nck) cp[j] = s;
    }
    endst[g] = s;
}

__device__ __forceinline__ bool same_state(const PllChannelState& a, const PllChannelState& b) {
    const unsigned* x = reinterpret_cast<const unsigned*>(&a);
    const unsigned* y = reinterpret_cast<const unsigned*>(&b);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < (int)(offsetof(PllChannelState, pad) / sizeof(float)); ++i) eq &= x[i] == y[i];
    return eq;
}

// Parallel re-run of the segments whose warm-up missed.  A segment's true start state is the
// previous segment's end state, and pass 1's end state of the previous segment IS that state
// whenever the previous segment ended on the true trajectory (its guess was right, or its
// trajectory met the true one before its end -- the common case).  So every segment whose guess
// differs from pass 1's end of its predecessor is re-run at once, one lane each, from that end
// state, until it meets its own pass-1 trajectory at a checkpoint (rstop = +intervals run) or
// to its end (rstop = -intervals, end state in end2).  pll_fix_kernel then only checks, per
// channel and in order, that each re-run started from the true state; where one did not
// (its predecessor's pass-1 end was not true), it recomputes that segment serially as before.
template <bool U8, int LID, int OID, int KID, int MODE, bool VEC>
__global__ __launch_bounds__(kPllBlock) void pll_refix_kernel(
    PllDevParams p, const void* __restrict__ in_, long ld_in, long n, float* __restrict__ out,
    uint8_t* __restrict__ locked, long ld_out, long seg, long warm, long nseg,
    const PllChannelState* __restrict__ guess, const PllChannelState* __restrict__ endst, long ck,
    const PllChannelState* __restrict__ ckpt, int* __restrict__ rstop,
    PllChannelState* __restrict__ end2) {
    own_simd();
    const long g = (long)blockIdx.x * kPllBlock + threadIdx.x;
    if (g < p.nch || g >= p.nch * nseg) return;  // segment 0 starts from the carried state
    const long ch = g % p.nch, sg = g / p.nch;
    const long t0 = sg * seg, t1 = t0 + seg < n ? t0 + seg : n;
    if (t0 <= warm || same_state(guess[g], endst[g - p.nch])) {
        rstop[g] = 0;
        return;
    }
    const PllLane<LID, OID, KID, MODE> ln(p);
    const void* row = static_cast<const char*>(in_) + ch * ld_in * (U8 ? 2 : 8);
    PllChannelState t = endst[g - p.nch];
    const long nck = seg / ck;
    const PllChannelState* __restrict__ cp = ckpt + g * (nck - 1);
    int k = 0;
    bool met = false;
    for (long j = 0; j < nck && !met; ++j) {
        const long a = t0 + j * ck, b = j + 1 < nck ? (a + ck < t1 ? a + ck : t1) : t1;
        if (a >= b) break;
        pll_run<U8, VEC, true>(ln, t, row, a, b, out + ch * ld_out, locked + ch * ld_out);
        ++k;
        met = j + 1 < nck && same_state(cp[j], t);
    }
    rstop[g] = met ? k : -k;
    if (!met) end2[g] = t;
}

template <bool U8, int LID, int OID, int KID, int MODE, bool VEC>
__global__ __launch_bounds__(kPllBlock) void pll_fix_kernel(
    PllDevParams p, const void* __restrict__ in_, long ld_in, long n, float* __restrict__ out,
    uint8_t* __restrict__ locked, long ld_out, PllChannelState* __restrict__ state, long seg,
    long warm, long nseg, const PllChannelState* __restrict__ guess,
    const PllChannelState* __restrict__ endst, unsigned long long* __restrict__ recomputed, long ck,
    const PllChannelState* __restrict__ ckpt, const int* __restrict__ rstop,
    const PllChannelState* __restrict__ end2) {
    own_simd();
    const long ch = (long)blockIdx.x * kPllBlock + threadIdx.x;
    if (ch >= p.nch) return;
    const PllLane<LID, OID, KID, MODE> ln(p);
    const void* row = static_cast<const char*>(in_) + ch * ld_in * (U8 ? 2 : 8);
    PllChannelState t = endst[ch];  // segment 0 started from the carried state: exact
    for (long sg = 1; sg < nseg; ++sg) {
        const long t0 = sg * seg, t1 = t0 + seg < n ? t0 + seg : n;
        const long g = sg * p.nch + ch;
        const bool hit = t0 <= warm || same_state(guess[g], t);
        const int rs = rstop[g];
        if (hit && rs == 0) {  // pass 1 ran from the true state and nothing overwrote it
            t = endst[g];
            continue;
        }
        if (!hit) {
            atomicAdd(recomputed, 1ull);
            if (rs != 0 && same_state(endst[g - p.nch], t)) {  // re-run from the true state: exact
                t = rs > 0 ? endst[g] : end2[g];
                continue;
            }
        }
        // the warm-up did not reach the true state and no re-run started from it, or a re-run
        // from a wrong state (its predecessor's pass-1 end) overwrote outputs of a segment whose
        // guess was right: this segment again from the true state, up to the first checkpoint
        // its trajectory meets (from there on it is exact) and at least over the overwritten
        // intervals
        const long nck = seg / ck, over = rs < 0 ? -rs : rs;
        const PllChannelState* __restrict__ cp = ckpt + g * (nck - 1);
        bool met = false;
        for (long j = 0; j < nck && !(met && j >= over); ++j) {
            const long a = t0 + j * ck, b = j + 1 < nck ? (a + ck < t1 ? a + ck : t1) : t1;
            if (a >= b) break;
            pll_run<U8, VEC, true>(ln, t, row, a, b, out + ch * ld_out, locked + ch * ld_out);
            met = j + 1 < nck && same_state(cp[j], t);
        }
        if (met) t = endst[g];
    }
    state[ch] = t;
}

// Output modes 0 and 1 with vector rows (configs[3]'s 1024 channels, main.rs's single
// stream and its stereo pilot):
// the lock and output filters are off the loop-carried chain (pll.rs:78-79 read c.re and
// phasedif, nothing feeds back), yet inside one wave they take issue slots from it -- and a
// wave alone on its SIMD is issue-bound.  So a 128-lane workgroup runs the chain on wave 0
// and the two filters, the output select and the stores on wave 1 (another SIMD): wave 0
// hands (c.re, phasedif) of each 8-sample chunk over through a two-slot LDS ring, one
// workgroup barrier per chunk.  Every operation is the same as in pll_kernel (bit-identical).
template <bool U8, int LID, int OID, int KID, int MODE>
__global__ __launch_bounds__(2 * kPllBlock) void pll_split_kernel(
    PllDevParams p, const void* __restrict__ in_, long ld_in, long n, float* __restrict__ out,
    uint8_t* __restrict__ locked, long ld_out, PllChannelState* __restrict__ state) {
    __shared__ float2 ring[2][kChunk][kPllBlock];
    // output mode 1 (the stereo pilot) also needs the input's real part and the new NCO value
    __shared__ float4 ring1[MODE == 1 ? 2 : 1][kChunk][kPllBlock];
    __shared__ float fst[8][kPllBlock];  // the helper's filter states, handed back at the end
    own_simd();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // lanes past the last channel run a copy of the last channel and store nothing (every
    // lane takes part in the per-chunk barriers)
    const bool on = (long)blockIdx.x * kPllBlock + lane < p.nch;
    const long ch = on ? (long)blockIdx.x * kPllBlock + lane : p.nch - 1;
    PllChannelState s = state[ch];
    const float2* __restrict__ xf = static_cast<const float2*>(in_) + ch * ld_in;
    const unsigned short* __restrict__ xu = static_cast<const unsigned short*>(in_) + ch * ld_in;
    auto cvt = [](unsigned w) -> float2 {
        return make_float2(((float)(w & 255u) - 128.0f) / 128.0f, ((float)((w >> 8) & 255u) - 128.0f) / 128.0f);
    };
    float* __restrict__ y = out + ch * ld_out;
    uint8_t* __restrict__ lk = locked + ch * ld_out;
    const Bq L = {p.loopc[0], p.loopc[1], p.loopc[2], p.loopc[3], p.loopc[4]};
    const Bq O = {p.outc[0], p.outc[1], p.outc[2], p.outc[3], p.outc[4]};
    const Bq K = {p.lockc[0], p.lockc[1], p.lockc[2], p.lockc[3], p.lockc[4]};
    const bool loop_id = LID == 2 ? p.loop_ident != 0 : LID == 1;
    const bool out_id = OID == 2 ? p.out_ident != 0 : OID == 1;
    const bool lock_id = KID == 2 ? p.lock_ident != 0 : KID == 1;
    constexpr float kTwoPi = 2.0f * 3.14159265358979323846f;
    // the loop-carried part of Pll::apply (pll.rs:71-76): returns (c.re, phasedif)
    auto chain = [&](float2 v) -> float2 {
        const float cjr = s.vr, cji = -s.vi;
        const float cr = v.x * cjr - v.y * cji;
        const float ci = v.x * cji + v.y * cjr;
        float lr = cr, li = ci;
        if (!loop_id) {
            float orr = 0.0f, oi = 0.0f;
            orr += cr * L.b0;      oi += ci * L.b0;
            orr += s.lx1r * L.b1;  oi += s.lx1i * L.b1;
            orr += s.lx2r * L.b2;  oi += s.lx2i * L.b2;
            orr += s.ly1r * L.na1; oi += s.ly1i * L.na1;
            orr += s.ly2r * L.na2; oi += s.ly2i * L.na2;
            s.lx2r = s.lx1r; s.lx1r = cr; s.ly2r = s.ly1r; s.ly1r = orr;
            s.lx2i = s.lx1i; s.lx1i = ci; s.ly2i = s.ly1i; s.ly1i = oi;
            lr = orr;
            li = oi;
        }
        const float phasedif = sdr_atan2f_bfx(li, lr) * p.gain;
        float nph = s.nphase + (p.reference + phasedif);
        nph = nph - truncf(nph);
        s.nphase = nph;
        const float phase = kTwoPi * nph;
        float sn, cs;
        sdr_sincosf_bf2(phase, &sn, &cs);
        s.vr = 1.0f * cs;
        s.vi = 1.0f * sn;
        return make_float2(cr, phasedif);
    };
    // pll.rs:78-84; output mode 1: src/main.rs:58-66 from (v.x, new value) in w
    auto filters = [&](float2 cp, float4 w, float& ov, uint8_t& lv) {
        const float cr = cp.x, phasedif = cp.y;
        const float lockv = lock_id ? cr : bq_real(K, cr, s.kx1, s.kx2, s.ky1, s.ky2);
        const float o = out_id ? phasedif * p.rate
                               : bq_real(O, phasedif * p.rate, s.ox1, s.ox2, s.oy1, s.oy2);
        const bool lockd = lockv > 0.01f;
        lv = lockd ? 1 : 0;
        if constexpr (MODE == 1) {
            const float vr = w.y, vi = w.z;
            const float wr = vr * vr - vi * vi;
            const float wi = vr * vi + vi * vr;
            const float nrm = wr * wr + wi * wi;
            const float dre = w.x * wr / nrm;
            ov = lockd ? dre * 0.5f : 0.0f;
        } else {
            ov = lockd ? o : 0.0f;
        }
    };
    using RawT = std::conditional_t<U8, uint4, float4>;
    constexpr int NR = U8 ? 1 : kChunk / 2;
    const long nchunks = n / kChunk, nfull = nchunks * kChunk;
    if (wv == 0) {  // the chain
        RawT raw[NR];
        auto ldc = [&](long i) {
            const RawT* q = reinterpret_cast<const RawT*>(U8 ? (const void*)(xu + i) : (const void*)(xf + i));
#pragma unroll
            for (int r = 0; r < NR; ++r) raw[r] = q[r];
        };
        auto sample = [&](int k) -> float2 {
            if constexpr (U8) {
                const unsigned w = (&raw[0].x)[k >> 1];
                return cvt((k & 1) ? (w >> 16) : (w & 0xffffu));
            } else {
                const float4 r = raw[k >> 1];
                return (k & 1) ? make_float2(r.z, r.w) : make_float2(r.x, r.y);
            }
        };
        float2 buf[kChunk];
        if (nchunks > 0) {
            ldc(0);
#pragma unroll
            for (int k = 0; k < kChunk; ++k) buf[k] = sample(k);
        }
        for (long c = 0; c < nchunks; ++c) {
            float2 cur[kChunk];
#pragma unroll
            for (int k = 0; k < kChunk; ++k) cur[k] = buf[k];
            if (c + 1 < nchunks) {
                ldc((c + 1) * kChunk);
#pragma unroll
                for (int k = 0; k < kChunk; ++k) buf[k] = sample(k);
            }
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                ring[c & 1][k][lane] = chain(cur[k]);
                if constexpr (MODE == 1) ring1[c & 1][k][lane] = make_float4(cur[k].x, s.vr, s.vi, 0.0f);
            }
            __syncthreads();  // chunk c published; the helper is done with chunk c - 1
        }
    } else {  // the filters, the output select and the stores
        for (long c = 0; c < nchunks; ++c) {
            __syncthreads();
            float ov[kChunk];
            uint8_t lv[kChunk];
#pragma unroll
            for (int k = 0; k < kChunk; ++k)
                filters(ring[c & 1][k][lane], MODE == 1 ? ring1[MODE == 1 ? (c & 1) : 0][k][lane] : float4{},
                        ov[k], lv[k]);
            if (on) {
                const long i = c * kChunk;
                float4* yo = reinterpret_cast<float4*>(y + i);
                yo[0] = make_float4(ov[0], ov[1], ov[2], ov[3]);
                yo[1] = make_float4(ov[4], ov[5], ov[6], ov[7]);
                uint2 pk;
                pk.x = lv[0] | (lv[1] << 8) | (lv[2] << 16) | ((unsigned)lv[3] << 24);
                pk.y = lv[4] | (lv[5] << 8) | (lv[6] << 16) | ((unsigned)lv[7] << 24);
                *reinterpret_cast<uint2*>(lk + i) = pk;
            }
        }
        fst[0][lane] = s.kx1; fst[1][lane] = s.kx2; fst[2][lane] = s.ky1; fst[3][lane] = s.ky2;
        fst[4][lane] = s.ox1; fst[5][lane] = s.ox2; fst[6][lane] = s.oy1; fst[7][lane] = s.oy2;
    }
    __syncthreads();
    if (wv != 0) return;
    // wave 0: the filter states back, the ragged tail (whole steps), the channel state
    s.kx1 = fst[0][lane]; s.kx2 = fst[1][lane]; s.ky1 = fst[2][lane]; s.ky2 = fst[3][lane];
    s.ox1 = fst[4][lane]; s.ox2 = fst[5][lane]; s.oy1 = fst[6][lane]; s.oy2 = fst[7][lane];
    if (!on) return;
    for (long i = nfull; i < n; ++i) {
        float o;
        uint8_t l;
        const float2 v = U8 ? cvt(xu[i]) : xf[i];
        const float2 cp = chain(v);
        filters(cp, make_float4(v.x, s.vr, s.vi, 0.0f), o, l);
        y[i] = o;
        lk[i] = l;
    }
    state[ch] = s;
}

template <bool U8, int LID, int OID, int KID, int MODE>
void launch_cfg(const PllDevParams& p, const void* in, long ld_in, long n, float* out,
                uint8_t* locked, long ld_out, PllChannelState* state, const PllSpec& spec,
                hipStream_t s) {
    const long nblk = (p.nch + kPllBlock - 1) / kPllBlock;
    const size_t sb = U8 ? 2 : 8;
    const bool vec = (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (ld_in * sb) % 16 == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (ld_out % 8) == 0 &&
                     (reinterpret_cast<uintptr_t>(locked) & 7) == 0;
    if (spec.seg > 0 && n > spec.seg) {  // time-parallel segments (seg, warm multiples of kChunk)
        const long nseg = (n + spec.seg - 1) / spec.seg;
        const long sblk = (p.nch * nseg + kPllBlock - 1) / kPllBlock;
#define SDRGPU_PLL_SEG(V)                                                                          \
        if (spec.phase_ev) (void)hipEventRecord(spec.phase_ev[0], s);                              \
        hipLaunchKernelGGL((pll_seg_kernel<U8, LID, OID, KID, MODE, V>), dim3((unsigned)sblk),      \
                           dim3(kPllBlock), 0, s, p, in, ld_in, n, out, locked, ld_out, state,       \
                           spec.seg, spec.warm, nseg, spec.guess, spec.end, spec.ck, spec.ckpt);    \
        if (spec.phase_ev) (void)hipEventRecord(spec.phase_ev[1], s);                              \
        hipLaunchKernelGGL((pll_refix_kernel<U8, LID, OID, KID, MODE, V>), dim3((unsigned)sblk),    \
                           dim3(kPllBlock), 0, s, p, in, ld_in, n, out, locked, ld_out, spec.seg,   \
                           spec.warm, nseg, spec.guess, spec.end, spec.ck, spec.ckpt, spec.rstop,   \
                           spec.end2);                                                              \
        if (spec.phase_ev) (void)hipEventRecord(spec.phase_ev[2], s);                              \
        hipLaunchKernelGGL((pll_fix_kernel<U8, LID, OID, KID, MODE, V>), dim3((unsigned)nblk),      \
                           dim3(kPllBlock), 0, s, p, in, ld_in, n, out, locked, ld_out, state,       \
                           spec.seg, spec.warm, nseg, spec.guess, spec.end, spec.recomputed,        \
                           spec.ck, spec.ckpt, spec.rstop, spec.end2);                              \
        if (spec.phase_ev) (void)hipEventRecord(spec.phase_ev[3], s)
        if (vec) { SDRGPU_PLL_SEG(true); } else { SDRGPU_PLL_SEG(false); }
#undef SDRGPU_PLL_SEG
        return;
    }
    if (vec && (MODE == 0 || MODE == 1))
        hipLaunchKernelGGL((pll_split_kernel<U8, LID, OID, KID, MODE>), dim3((unsigned)nblk),
                           dim3(2 * kPllBlock), 0, s, p, in, ld_in, n, out, locked, ld_out, state);
    else if (vec)
        hipLaunchKernelGGL((pll_kernel<U8, LID, OID, KID, MODE, true>), dim3((unsigned)nblk),
                           dim3(kPllBlock), 0, s, p, in, ld_in, n, out, locked, ld_out, state);
    else
        hipLaunchKernelGGL((pll_kernel<U8, LID, OID, KID, MODE, false>), dim3((unsigned)nblk),
                           dim3(kPllBlock), 0, s, p, in, ld_in, n, out, locked, ld_out, state);
}

template <bool U8>
void launch_any(const PllDevParams& p, const void* in, long ld_in, long n, float* out,
                uint8_t* locked, long ld_out, PllChannelState* state, const PllSpec& spec,
                hipStream_t s) {
    const int l = p.loop_ident, o = p.out_ident, k = p.lock_ident, m = p.out_mode;
    if (!l && o && !k && m == 0)            // src/main.rs:41-46
        launch_cfg<U8, 0, 1, 0, 0>(p, in, ld_in, n, out, locked, ld_out, state, spec, s);
    else if (!l && !o && !k && m == 0)      // examples/pll.rs:9-15
        launch_cfg<U8, 0, 0, 0, 0>(p, in, ld_in, n, out, locked, ld_out, state, spec, s);
    else if (!l && !o && !k && m == 1)      // the stereo pilot, src/main.rs:55-66
        launch_cfg<U8, 0, 0, 0, 1>(p, in, ld_in, n, out, locked, ld_out, state, spec, s);
    else
        launch_cfg<U8, 2, 2, 2, 2>(p, in, ld_in, n, out, locked, ld_out, state, spec, s);
}

}  // namespace

// The device forms of the libm functions the PLL chain calls (Pll::apply's arg() and
// from_polar, src/filter/pll.rs:72-76): fn 0 = sdr_atan2f_bfx(a, b) (y = a, x = b), fn 1 =
// sdr_sincosf_bf2(a).  Test-only (sdrgpu_debug_libm): the same inlined code as the kernels
// above, so special operands (zeros, subnormals, infinities, NaN), the wave ballot that skips
// their selects and the f64 / reciprocal divisions can be compared with glibc on the device.
__global__ __launch_bounds__(256) void libm_debug_kernel(int fn, const float* __restrict__ a,
                                                         const float* __restrict__ b,
                                                         float* __restrict__ o0,
                                                         float* __restrict__ o1, long n) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (fn == 0) {
        o0[i] = sdr_atan2f_bfx(a[i], b[i]);
    } else {
        float sn, cs;
        sdr_sincosf_bf2(a[i], &sn, &cs);
        o0[i] = sn;
        o1[i] = cs;
    }
}

int libm_debug_launch(int fn, const float* a, const float* b, float* o0, float* o1, long n,
                      hipStream_t s) {
    if (n <= 0) return SDRGPU_OK;
    hipLaunchKernelGGL(libm_debug_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, fn,
                       a, b, o0, o1, n);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

int pll_launch(const PllDevParams& p, const void* in, long ld_in, long n, float* out,
               uint8_t* locked, long ld_out, PllChannelState* state, const PllSpec& spec,
               hipStream_t s) {
    if (n <= 0) return SDRGPU_OK;
    if (spec.seg > 0 && (spec.seg % kChunk || spec.warm % kChunk || !spec.guess || !spec.end ||
                         !spec.recomputed || spec.ck <= 0 || spec.ck % kChunk || spec.seg % spec.ck ||
                         (spec.seg / spec.ck > 1 && !spec.ckpt) || !spec.rstop || !spec.end2))
        return SDRGPU_ERR_INVALID;
    if (spec.seg > 0 && n > spec.seg)
        SDRGPU_HIP_TRY(hipMemsetAsync(spec.recomputed, 0, sizeof(unsigned long long), s));
    if (p.in_u8) launch_any<true>(p, in, ld_in, n, out, locked, ld_out, state, spec, s);
    else launch_any<false>(p, in, ld_in, n, out, locked, ld_out, state, spec, s);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

}  // namespace sdrgpu
