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
#include "common.hpp"

namespace sdrgpu {

struct BiquadState {
    float x1r, x1i, x2r, x2i, y1r, y1i, y2r, y2i;
};

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
__device__ __forceinline__ void own_simd() { asm volatile("" ::: "v255", "a255"); }

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

}  // namespace

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
