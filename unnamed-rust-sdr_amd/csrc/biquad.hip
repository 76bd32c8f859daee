// biquad.hip -- batched Biquad<C, f32>::apply (reference src/filter/biquad.rs:42-56) with the
// coefficients BiquadD::design produces (:83-155) or Identity (src/filter/simple.rs:3-19):
// one channel per lane, the DF1 state (x1, x2, y1, y2) in registers across the block,
// reference operation order
//     out = 0; out += x*b0; out += x1*b1; out += x2*b2; out += y1*na1; out += y2*na2
// with no FMA contraction (this file is built with -ffp-contract=off), so outputs are
// bit-identical to the reference's f32 arithmetic.  Complex samples: Convolve::accumulate
// for Complex<f32> * f32 (src/filter/convolve.rs:13-15) scales re and im separately, i.e.
// two real recurrences in the same order.  The recurrence is loop-carried, so a channel is
// serial; throughput comes from channels (64 per wave), and samples are prefetched 8 ahead.
#include "biquad_kernels.hpp"
#include "common.hpp"

namespace sdrgpu {

namespace {

constexpr int kBqBlock = 64;
constexpr int kBqChunk = 8;

__device__ __forceinline__ float bq_step(const float* c, float x, float& x1, float& x2, float& y1,
                                         float& y2) {
    float out = 0.0f;
    out += x * c[0];
    out += x1 * c[1];
    out += x2 * c[2];
    out += y1 * c[3];
    out += y2 * c[4];
    x2 = x1;
    x1 = x;
    y2 = y1;
    y1 = out;
    return out;
}

// A bit-exact recurrence built from packed-f32 VALU ops, like the PLL chain: each wave owns its
// SIMD (512 VGPRs claimed), so no MFMA wave of a concurrently running kernel can share it (the
// measured hazard is described at pll.hip's own_simd).  One channel per lane, so this costs
// nothing below 64 Ki channels.
__device__ __forceinline__ void own_simd() { claim_simd_whole(); }

template <bool CPLX>
__global__ __launch_bounds__(kBqBlock) void biquad_kernel(long nch, float b0, float b1, float b2,
                                                          float na1, float na2, int ident,
                                                          const float* __restrict__ in, long ld_in,
                                                          long n, float* __restrict__ out,
                                                          long ld_out, BiquadState* __restrict__ st) {
    own_simd();
    const long ch = (long)blockIdx.x * kBqBlock + threadIdx.x;
    if (ch >= nch) return;
    constexpr int W = CPLX ? 2 : 1;  // floats per sample
    const float c[5] = {b0, b1, b2, na1, na2};
    BiquadState s = st[ch];
    const float* __restrict__ x = in + ch * ld_in * W;
    float* __restrict__ y = out + ch * ld_out * W;
    long i = 0;
    for (; i + kBqChunk <= n; i += kBqChunk) {
        float v[kBqChunk * W];
#pragma unroll
        for (int k = 0; k < kBqChunk * W; ++k) v[k] = x[i * W + k];
#pragma unroll
        for (int k = 0; k < kBqChunk; ++k) {
            if (ident) continue;
            v[k * W] = bq_step(c, v[k * W], s.x1r, s.x2r, s.y1r, s.y2r);
            if (CPLX) v[k * W + 1] = bq_step(c, v[k * W + 1], s.x1i, s.x2i, s.y1i, s.y2i);
        }
#pragma unroll
        for (int k = 0; k < kBqChunk * W; ++k) y[i * W + k] = v[k];
    }
    for (; i < n; ++i) {
        float vr = x[i * W], vi = CPLX ? x[i * W + 1] : 0.f;
        if (!ident) {
            vr = bq_step(c, vr, s.x1r, s.x2r, s.y1r, s.y2r);
            if (CPLX) vi = bq_step(c, vi, s.x1i, s.x2i, s.y1i, s.y2i);
        }
        y[i * W] = vr;
        if (CPLX) y[i * W + 1] = vi;
    }
    st[ch] = s;
}

// Samples [a, b) of one channel through the recurrence (the kernel above, on a sub-range):
// STORE writes the outputs, otherwise only the state advances (a warm-up).
template <bool CPLX, bool STORE>
__device__ __forceinline__ void bq_run(const float (&c)[5], BiquadState& s, const float* __restrict__ x,
                                       float* __restrict__ y, long a, long b) {
    constexpr int W = CPLX ? 2 : 1;
    long i = a;
    for (; i + kBqChunk <= b; i += kBqChunk) {
        float v[kBqChunk * W];
#pragma unroll
        for (int k = 0; k < kBqChunk * W; ++k) v[k] = x[i * W + k];
#pragma unroll
        for (int k = 0; k < kBqChunk; ++k) {
            v[k * W] = bq_step(c, v[k * W], s.x1r, s.x2r, s.y1r, s.y2r);
            if (CPLX) v[k * W + 1] = bq_step(c, v[k * W + 1], s.x1i, s.x2i, s.y1i, s.y2i);
        }
        if constexpr (STORE) {
#pragma unroll
            for (int k = 0; k < kBqChunk * W; ++k) y[i * W + k] = v[k];
        }
    }
    for (; i < b; ++i) {
        float vr = bq_step(c, x[i * W], s.x1r, s.x2r, s.y1r, s.y2r);
        float vi = CPLX ? bq_step(c, x[i * W + 1], s.x1i, s.x2i, s.y1i, s.y2i) : 0.f;
        if constexpr (STORE) {
            y[i * W] = vr;
            if (CPLX) y[i * W + 1] = vi;
        }
    }
}

// Time-parallel blocks, the PLL's scheme (pll.hip) on a linear recurrence:
// a stable biquad forgets its output history geometrically, so a copy started `warm` samples
// early from zero output history (x1 / x2 are the block's own inputs, exact) reaches the true
// (y1, y2) bit for bit, typically within a few pole time constants.  bq_seg_kernel: one lane
// per channel-segment, warm-up (state only), the guess at the segment start, the segment's
// outputs with checkpoints every ck samples, its end state.  bq_refix_kernel: every segment
// whose guess differs from its predecessor's pass-1 end is re-run from that end state, up to
// the checkpoint where it meets its own pass-1 trajectory.  bq_fix_kernel: per channel, in
// order, with the true state: a segment whose guess was true and was not overwritten, or whose
// re-run started from the true state, is exact; any other is recomputed serially.  Every
// output is the serial recurrence's.
__device__ __forceinline__ bool bq_same(const BiquadState& a, const BiquadState& b) {
    return __float_as_uint(a.y1r) == __float_as_uint(b.y1r) && __float_as_uint(a.y2r) == __float_as_uint(b.y2r) &&
           __float_as_uint(a.y1i) == __float_as_uint(b.y1i) && __float_as_uint(a.y2i) == __float_as_uint(b.y2i) &&
           __float_as_uint(a.x1r) == __float_as_uint(b.x1r) && __float_as_uint(a.x2r) == __float_as_uint(b.x2r) &&
           __float_as_uint(a.x1i) == __float_as_uint(b.x1i) && __float_as_uint(a.x2i) == __float_as_uint(b.x2i);
}

template <bool CPLX>
__global__ __launch_bounds__(kBqBlock) void bq_seg_kernel(long nch, float b0, float b1, float b2,
                                                          float na1, float na2,
                                                          const float* __restrict__ in, long ld_in,
                                                          long n, float* __restrict__ out, long ld_out,
                                                          const BiquadState* __restrict__ st,
                                                          BqSpec sp) {
    own_simd();
    const long g = (long)blockIdx.x * kBqBlock + threadIdx.x;
    if (g >= nch * sp.nseg) return;
    constexpr int W = CPLX ? 2 : 1;
    const long ch = g % nch, sg = g / nch;
    const long t0 = sg * sp.seg, t1 = t0 + sp.seg < n ? t0 + sp.seg : n;
    long tw = t0 > sp.warm ? t0 - sp.warm : 0;
    if (tw < 2) tw = 0;  // a warm-up start needs the two inputs before it
    const float c[5] = {b0, b1, b2, na1, na2};
    const float* __restrict__ x = in + ch * ld_in * W;
    float* __restrict__ y = out + ch * ld_out * W;
    BiquadState s{};
    if (tw == 0) {
        s = st[ch];
    } else {  // zero output history; the input history is the block's own samples
        s.x1r = x[(tw - 1) * W];
        s.x2r = x[(tw - 2) * W];
        if (CPLX) {
            s.x1i = x[(tw - 1) * W + 1];
            s.x2i = x[(tw - 2) * W + 1];
        }
    }
    bq_run<CPLX, false>(c, s, x, y, tw, t0);
    sp.guess[g] = s;
    const long nck = sp.seg / sp.ck;
    BiquadState* __restrict__ cp = sp.ckpt + g * (nck - 1);
    for (long j = 0; j < nck; ++j) {
        const long a = t0 + j * sp.ck, b = j + 1 < nck ? (a + sp.ck < t1 ? a + sp.ck : t1) : t1;
        if (a >= b) break;
        bq_run<CPLX, true>(c, s, x, y, a, b);
        if (j + 1 < nck) cp[j] = s;
    }
    sp.end[g] = s;
}

template <bool CPLX>
__global__ __launch_bounds__(kBqBlock) void bq_refix_kernel(long nch, float b0, float b1, float b2,
                                                            float na1, float na2,
                                                            const float* __restrict__ in, long ld_in,
                                                            long n, float* __restrict__ out, long ld_out,
                                                            BqSpec sp) {
    own_simd();
    const long g = (long)blockIdx.x * kBqBlock + threadIdx.x;
    if (g < nch || g >= nch * sp.nseg) return;  // segment 0 starts from the carried state
    constexpr int W = CPLX ? 2 : 1;
    const long ch = g % nch, sg = g / nch;
    const long t0 = sg * sp.seg, t1 = t0 + sp.seg < n ? t0 + sp.seg : n;
    if (t0 - sp.warm < 2 || bq_same(sp.guess[g], sp.end[g - nch])) {
        sp.rstop[g] = 0;
        return;
    }
    const float c[5] = {b0, b1, b2, na1, na2};
    const float* __restrict__ x = in + ch * ld_in * W;
    float* __restrict__ y = out + ch * ld_out * W;
    BiquadState t = sp.end[g - nch];
    const long nck = sp.seg / sp.ck;
    const BiquadState* __restrict__ cp = sp.ckpt + g * (nck - 1);
    int k = 0;
    bool met = false;
    for (long j = 0; j < nck && !met; ++j) {
        const long a = t0 + j * sp.ck, b = j + 1 < nck ? (a + sp.ck < t1 ? a + sp.ck : t1) : t1;
        if (a >= b) break;
        bq_run<CPLX, true>(c, t, x, y, a, b);
        ++k;
        met = j + 1 < nck && bq_same(cp[j], t);
    }
    sp.rstop[g] = met ? k : -k;
    if (!met) sp.end2[g] = t;
}

template <bool CPLX>
__global__ __launch_bounds__(kBqBlock) void bq_fix_kernel(long nch, float b0, float b1, float b2,
                                                          float na1, float na2,
                                                          const float* __restrict__ in, long ld_in,
                                                          long n, float* __restrict__ out, long ld_out,
                                                          BiquadState* __restrict__ st, BqSpec sp) {
    own_simd();
    const long ch = (long)blockIdx.x * kBqBlock + threadIdx.x;
    if (ch >= nch) return;
    constexpr int W = CPLX ? 2 : 1;
    const float c[5] = {b0, b1, b2, na1, na2};
    const float* __restrict__ x = in + ch * ld_in * W;
    float* __restrict__ y = out + ch * ld_out * W;
    BiquadState t = sp.end[ch];  // segment 0 started from the carried state: exact
    for (long sg = 1; sg < sp.nseg; ++sg) {
        const long t0 = sg * sp.seg, t1 = t0 + sp.seg < n ? t0 + sp.seg : n;
        const long g = sg * nch + ch;
        const bool hit = t0 - sp.warm < 2 || bq_same(sp.guess[g], t);
        const int rs = sp.rstop[g];
        if (hit && rs == 0) {
            t = sp.end[g];
            continue;
        }
        if (!hit) {
            atomicAdd(sp.recomputed, 1ull);
            if (rs != 0 && bq_same(sp.end[g - nch], t)) {  // re-run from the true state: exact
                t = rs > 0 ? sp.end[g] : sp.end2[g];
                continue;
            }
        }
        // recompute from the true state up to the first checkpoint it meets, and at least over
        // the intervals a re-run from a wrong state overwrote
        const long nck = sp.seg / sp.ck, over = rs < 0 ? -rs : rs;
        const BiquadState* __restrict__ cp = sp.ckpt + g * (nck - 1);
        bool met = false;
        for (long j = 0; j < nck && !(met && j >= over); ++j) {
            const long a = t0 + j * sp.ck, b = j + 1 < nck ? (a + sp.ck < t1 ? a + sp.ck : t1) : t1;
            if (a >= b) break;
            bq_run<CPLX, true>(c, t, x, y, a, b);
            met = j + 1 < nck && bq_same(cp[j], t);
        }
        if (met) t = sp.end[g];
    }
    st[ch] = t;
}

}  // namespace

int biquad_tp_launch(bool cplx, long nch, const float* c, const void* in, long ld_in, long n,
                     void* out, long ld_out, BiquadState* state, const BqSpec& sp, hipStream_t s) {
    if (nch <= 0 || n <= 0) return SDRGPU_OK;
    if (sp.seg <= 0 || sp.seg % kBqChunk || sp.ck <= 0 || sp.ck % kBqChunk || sp.seg % sp.ck ||
        sp.nseg != ceil_div(n, sp.seg) || sp.nseg < 2 || !sp.guess || !sp.end || !sp.end2 ||
        !sp.rstop || !sp.recomputed || (sp.seg / sp.ck > 1 && !sp.ckpt))
        return SDRGPU_ERR_INVALID;
    SDRGPU_HIP_TRY(hipMemsetAsync(sp.recomputed, 0, sizeof(unsigned long long), s));
    const dim3 gs((unsigned)ceil_div(nch * sp.nseg, kBqBlock)), gc((unsigned)ceil_div(nch, kBqBlock)), b(kBqBlock);
    const float* x = static_cast<const float*>(in);
    float* y = static_cast<float*>(out);
#define SDRGPU_BQ_TP(CP)                                                                          \
    hipLaunchKernelGGL(bq_seg_kernel<CP>, gs, b, 0, s, nch, c[0], c[1], c[2], c[3], c[4], x, ld_in, \
                       n, y, ld_out, state, sp);                                                  \
    hipLaunchKernelGGL(bq_refix_kernel<CP>, gs, b, 0, s, nch, c[0], c[1], c[2], c[3], c[4], x,    \
                       ld_in, n, y, ld_out, sp);                                                  \
    hipLaunchKernelGGL(bq_fix_kernel<CP>, gc, b, 0, s, nch, c[0], c[1], c[2], c[3], c[4], x, ld_in, \
                       n, y, ld_out, state, sp)
    if (cplx) {
        SDRGPU_BQ_TP(true);
    } else {
        SDRGPU_BQ_TP(false);
    }
#undef SDRGPU_BQ_TP
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

int biquad_launch(bool cplx, long nch, const float* c, int ident, const void* in, long ld_in,
                  long n, void* out, long ld_out, BiquadState* state, hipStream_t s) {
    if (nch <= 0 || n <= 0) return SDRGPU_OK;
    const dim3 g((unsigned)ceil_div(nch, kBqBlock)), b(kBqBlock);
    if (cplx)
        hipLaunchKernelGGL(biquad_kernel<true>, g, b, 0, s, nch, c[0], c[1], c[2], c[3], c[4],
                           ident, static_cast<const float*>(in), ld_in, n,
                           static_cast<float*>(out), ld_out, state);
    else
        hipLaunchKernelGGL(biquad_kernel<false>, g, b, 0, s, nch, c[0], c[1], c[2], c[3], c[4],
                           ident, static_cast<const float*>(in), ld_in, n,
                           static_cast<float*>(out), ld_out, state);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

}  // namespace sdrgpu
