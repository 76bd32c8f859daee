// fir_exact.hpp -- the reference's FIR sum per output, for tiles / blocks holding inf or NaN
// samples (fir_direct.hip, fir_direct2.hip, fir_os.hip, fir_mfma.hip; fir_mxh.hip has its own).
#pragma once

#include "fir_kernels.hpp"

namespace sdrgpu {

// -------- inf / NaN samples: the reference's own sum --------
// The fast kernels spread a non-finite sample beyond the K outputs whose window holds it in the
// reference: zero-padded taps multiply samples outside an output's window (0 x NaN = NaN), an
// FFT block mixes all of its samples, a scaled split has no scale for it.  Their non-finite
// outputs are recomputed with fir_exact_output: Fir::apply's sum as written
// (fir.rs:28-30, convolve.rs:13-15): acc = 0; acc += x[g - k] * h[k] for k = 0 .. K-1, the
// num-complex product, no FMA, x[< 0] from the carried history.  Non-finite outputs are then
// exactly the reference's.
// The arithmetic is written as VOP2 instructions: plain C++ lets the compiler pair the re / im
// halves into packed-f32 ops, and a packed product read by the next packed op without a wait
// state went wrong in lanes 48-63 beside another wave's MFMAs (DESIGN.md 3.6,
// profiles/r06_pkfault.txt).  The MFMA kernels that call these need that; the others lose
// nothing that matters on a path only inf / NaN samples take.  IEEE-exact, no contraction.
__device__ __forceinline__ float vop2_mul(float a, float b) {
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vop2_add(float a, float b) {
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vop2_sub(float a, float b) {
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float exact_prod(float x, float h) { return vop2_mul(x, h); }
__device__ __forceinline__ c64 exact_prod(c64 x, float h) {
    return make_float2(vop2_mul(x.x, h), vop2_mul(x.y, h));
}
__device__ __forceinline__ c64 exact_prod(c64 x, c64 h) {
    return make_float2(vop2_sub(vop2_mul(x.x, h.x), vop2_mul(x.y, h.y)),
                       vop2_add(vop2_mul(x.x, h.y), vop2_mul(x.y, h.x)));
}
__device__ __forceinline__ void exact_add(float& a, float b) { a = vop2_add(a, b); }
__device__ __forceinline__ void exact_add(c64& a, c64 b) {
    a.x = vop2_add(a.x, b.x);
    a.y = vop2_add(a.y, b.y);
}
constexpr int kExactBatch = 8;
// P: FirParams, or a kernel's own parameter block with the same i0 / n_in / K / D / taps_pm / tpp
template <typename TS, typename TT, typename P>
__device__ __forceinline__ TS fir_exact_output(const P& p, const TS* __restrict__ in,
                                               const TS* __restrict__ hist, long m) {
    const TT* __restrict__ taps = static_cast<const TT*>(p.taps_pm);
    const long g = p.i0 + m * p.D;
    TS acc = zero_of<TS>();
    if (g - (p.K - 1) >= 0 && g < p.n_in) {
        // window inside this block: kExactBatch loads in flight per step, the sum still in k
        // order (an all-NaN stream takes this path for every output)
        const TS* __restrict__ xp = in + g;
        const int kb = p.K - p.K % kExactBatch;
#pragma unroll 1
        for (int k = 0; k < kb; k += kExactBatch) {
            TS xv[kExactBatch];
            TT hk[kExactBatch];
#pragma unroll
            for (int u = 0; u < kExactBatch; ++u) {
                xv[u] = xp[-(k + u)];
                hk[u] = taps[(long)((k + u) % p.D) * p.tpp + (k + u) / p.D];
            }
#pragma unroll
            for (int u = 0; u < kExactBatch; ++u) exact_add(acc, exact_prod(xv[u], hk[u]));
        }
#pragma unroll 1
        for (int k = kb; k < p.K; ++k)
            exact_add(acc, exact_prod(xp[-k], taps[(long)(k % p.D) * p.tpp + k / p.D]));
        return acc;
    }
#pragma unroll 1
    for (int k = 0; k < p.K; ++k) {
        const long j = g - k;
        TS x = zero_of<TS>();
        if (j >= 0) x = j < p.n_in ? in[j] : zero_of<TS>();
        else if (j >= -(long)(p.K - 1)) x = hist[j + (p.K - 1)];
        exact_add(acc, exact_prod(x, taps[(long)(k % p.D) * p.tpp + k / p.D]));
    }
    return acc;
}
__device__ __forceinline__ bool all_finite(float x) { return __builtin_isfinite(x); }
__device__ __forceinline__ bool all_finite(c64 x) { return __builtin_isfinite(x.x) & __builtin_isfinite(x.y); }
// A fast kernel's output that is not finite came from an inf / NaN sample somewhere in the
// kernel's reach for it (padded taps, the FFT block, the MFMA tile: finite samples never give a
// non-finite sum there short of f32 overflow, which the reference's sum then reproduces); it is
// replaced by the reference's sum, which is non-finite exactly where the reference's is.  Lanes
// with finite outputs skip the branch, so finite data pays two v_cmp_class per output.
template <typename TS, typename TT, typename P>
__device__ __forceinline__ TS fir_checked(const P& p, const TS* __restrict__ in,
                                          const TS* __restrict__ hist, long m, TS acc) {
    if (!all_finite(acc)) acc = fir_exact_output<TS, TT>(p, in, hist, m);
    return acc;
}
}  // namespace sdrgpu
