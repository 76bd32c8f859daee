// pll.hip -- batched PLL / FM demodulator (one channel per lane) for gfx950.
//
// Semantics: Pll::apply (reference src/filter/pll.rs:70-85) with BiquadD loop / output /
// lock filters (src/filter/biquad.rs:25-56, 83-155) or Identity (src/filter/simple.rs:3-19):
//   c = x * conj(v);  phasedif = arg(loop(c)) * gain;  nphase = fract(nphase + ref + phasedif)
//   v = from_polar(1, 2 pi nphase);  locked = lock(c.re);  out = output(phasedif * rate)
//   -> Some(out) if locked > 0.01 else None   (None written as 0.0, src/main.rs:49)
//
// The recurrence is serial and nonlinear (atan2 -> NCO -> sin/cos each sample), so it is
// latency-bound, not HBM- or FLOP-bound: the loop-carried chain is kept as
// short as the arithmetic allows -- each biquad's terms that only depend on past state are
// summed before the new input arrives, so only one FMA per filter sits on the chain -- and
// the next 8 samples of every lane are in flight while the current 8 are processed.
// Accurate ocml atan2f / sincosf are used (never the __sinf family) so the loop tracks the
// reference's glibc libm within a few ulp per sample.
#include <algorithm>

#include "common.hpp"
#include "pll_kernels.hpp"

namespace sdrgpu {

namespace {

constexpr int kPllBlock = 64;   // one wave: 64 channels
constexpr int kChunk = 8;       // samples per lane per pipeline stage

struct Bq {
    float b0, b1, b2, na1, na2;
};

__device__ __forceinline__ float bq_real(const Bq& c, float x, float& x1, float& x2, float& y1,
                                         float& y2) {
    // reference order: b0 x + b1 x1 + b2 x2 + na1 y1 + na2 y2 (biquad.rs:44-49); the past-
    // state part is formed first so the new input enters with a single FMA.
    const float pre = fmaf(c.na1, y1, fmaf(c.b2, x2, fmaf(c.na2, y2, c.b1 * x1)));
    const float out = fmaf(c.b0, x, pre);
    x2 = x1;
    x1 = x;
    y2 = y1;
    y1 = out;
    return out;
}

__global__ __launch_bounds__(kPllBlock) void pll_kernel(PllDevParams p, const float2* __restrict__ in,
                                                        long ld_in, long n, float* __restrict__ out,
                                                        uint8_t* __restrict__ locked, long ld_out,
                                                        PllChannelState* __restrict__ state) {
    const long ch = (long)blockIdx.x * kPllBlock + threadIdx.x;
    if (ch >= p.nch) return;
    PllChannelState s = state[ch];
    const float2* __restrict__ x = in + ch * ld_in;
    float* __restrict__ y = out + ch * ld_out;
    uint8_t* __restrict__ lk = locked + ch * ld_out;
    const Bq L = {p.loopc[0], p.loopc[1], p.loopc[2], p.loopc[3], p.loopc[4]};
    const Bq O = {p.outc[0], p.outc[1], p.outc[2], p.outc[3], p.outc[4]};
    const Bq K = {p.lockc[0], p.lockc[1], p.lockc[2], p.lockc[3], p.lockc[4]};
    constexpr float kTwoPi = 2.0f * 3.14159265358979323846f;  // 2.0 * f32::consts::PI

    float2 buf[kChunk];
    long i = 0;
    const long nfull = n / kChunk * kChunk;
    if (nfull > 0) {
#pragma unroll
        for (int k = 0; k < kChunk; ++k) buf[k] = x[k];
    }
    for (; i < n; i += kChunk) {
        const bool full = i < nfull;
        float2 cur[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) cur[k] = buf[k];
        if (!full) {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) cur[k] = (i + k < n) ? x[i + k] : make_float2(0.f, 0.f);
        } else if (i + kChunk < nfull) {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) buf[k] = x[i + kChunk + k];  // prefetch
        } else if (i + kChunk < n) {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) buf[k] = make_float2(0.f, 0.f);
        }
        float ov[kChunk];
        uint8_t lv[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            const float2 v = cur[k];
            // c = value * conj(self.value)  (pll.rs:71; num-complex Mul)
            const float cr = v.x * s.vr - v.y * (-s.vi);
            const float ci = v.x * (-s.vi) + v.y * s.vr;
            float lr = cr, li = ci;
            if (!p.loop_ident) {
                const float pr = fmaf(L.na1, s.ly1r, fmaf(L.b2, s.lx2r, fmaf(L.na2, s.ly2r, L.b1 * s.lx1r)));
                const float pi = fmaf(L.na1, s.ly1i, fmaf(L.b2, s.lx2i, fmaf(L.na2, s.ly2i, L.b1 * s.lx1i)));
                lr = fmaf(L.b0, cr, pr);
                li = fmaf(L.b0, ci, pi);
                s.lx2r = s.lx1r; s.lx1r = cr; s.ly2r = s.ly1r; s.ly1r = lr;
                s.lx2i = s.lx1i; s.lx1i = ci; s.ly2i = s.ly1i; s.ly1i = li;
            }
            const float phasedif = atan2f(li, lr) * p.gain;           // :72 arg()
            float nph = s.nphase + (p.reference + phasedif);           // :73
            nph = nph - truncf(nph);                                   // :74 fract()
            s.nphase = nph;
            float sn, cs;
            sincosf(kTwoPi * nph, &sn, &cs);                           // :75-76 from_polar
            s.vr = cs;
            s.vi = sn;
            const float lockv = p.lock_ident ? cr : bq_real(K, cr, s.kx1, s.kx2, s.ky1, s.ky2);  // :78
            const float o = p.out_ident ? phasedif * p.rate
                                        : bq_real(O, phasedif * p.rate, s.ox1, s.ox2, s.oy1, s.oy2);
            const bool lockd = lockv > 0.01f;                          // :80
            ov[k] = lockd ? o : 0.0f;
            lv[k] = lockd ? 1 : 0;
        }
        if (full) {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                y[i + k] = ov[k];
                lk[i + k] = lv[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < kChunk; ++k)
                if (i + k < n) {
                    y[i + k] = ov[k];
                    lk[i + k] = lv[k];
                }
        }
    }
    state[ch] = s;
}

}  // namespace

int pll_launch(const PllDevParams& p, const float2* in, long ld_in, long n, float* out,
               uint8_t* locked, long ld_out, PllChannelState* state, hipStream_t s) {
    if (n <= 0) return SDRGPU_OK;
    const long nblk = (p.nch + kPllBlock - 1) / kPllBlock;
    hipLaunchKernelGGL(pll_kernel, dim3((unsigned)nblk), dim3(kPllBlock), 0, s, p, in, ld_in, n, out,
                       locked, ld_out, state);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

}  // namespace sdrgpu
