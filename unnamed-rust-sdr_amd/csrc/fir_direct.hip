// fir_direct.hip -- direct-form streaming FIR / FIR-decimate for gfx950.
//
// Semantics: Fir::apply (reference src/filter/fir.rs:23-32) followed by Decimate
// (src/signal/adapters/mod.rs:30-37): y[m] = sum_k h[k] x[g_m - k], g_m = i0 + m*D, with
// x[<0] taken from the carried history and zero before the stream start.  Only kept
// outputs are computed.
//
// Design (MI355X): one workgroup (256 lanes = 4 wave64) produces NT = 256*R consecutive
// kept outputs of one channel.  The input span those outputs need (NT*D + ~K samples) is
// staged once into LDS with coalesced loads; the sample index is padded by one slot per
// 32 samples so that lanes, which read R*D-sample-strided windows, hit distinct banks.
// Each lane register-blocks R consecutive outputs.  The taps are split into D polyphase
// branches h_p[i] = h[p + i*D] (pre-arranged on the host, zero padded to a multiple of R,
// read through the scalar cache since they are wave-uniform): inside a branch, tap i+1 of
// output r uses the sample tap i of output r-1 used, so a sliding window of 2R registers
// does R*R MACs per R LDS reads.
// Roofline: 2*K (real taps) / 8*K (complex taps) flops per kept output; for K=255, D=4 on
// c64 it is FP32-VALU bound, see DESIGN.md.
#include <cstdlib>

#include "fir_exact.hpp"

namespace sdrgpu {

namespace {

constexpr int kBlock = 256;

__host__ __device__ __forceinline__ long lds_index(long s) { return s + (s >> 5); }

template <typename TS>
__device__ __forceinline__ TS fetch_stream(const TS* __restrict__ in, long n_in,
                                           const TS* __restrict__ hist, int K, long g) {
    if (g >= 0) return g < n_in ? in[g] : zero_of<TS>();
    if (g >= -(long)(K - 1)) return hist[g + (K - 1)];
    return zero_of<TS>();
}

// History carry: hist_next[j] = stream sample (n_in - (K-1) + j).  Run by one block per
// channel; reads hist/in only, writes the other ping-pong buffer, so no race with blocks
// still reading hist.
template <typename TS>
__device__ __forceinline__ void carry_history(const TS* __restrict__ in, long n_in,
                                              const TS* __restrict__ hist,
                                              TS* __restrict__ hist_next, int K) {
    for (int j = threadIdx.x; j < K - 1; j += blockDim.x) {
        long g = n_in - (long)(K - 1) + j;
        hist_next[j] = g >= 0 ? in[g] : hist[g + (K - 1)];
    }
}

template <typename TS, typename TT, int R>
__global__ __launch_bounds__(kBlock) void fir_direct_kernel(FirParams p) {
    extern __shared__ __align__(16) unsigned char smem_raw[];
    TS* lds = reinterpret_cast<TS*>(smem_raw);

    const long ch = blockIdx.y;
    const TS* __restrict__ in = static_cast<const TS*>(p.in) + ch * p.ld_in;
    const TS* __restrict__ hist = static_cast<const TS*>(p.hist) + ch * (long)(p.K - 1);
    TS* __restrict__ out = static_cast<TS*>(p.out) + ch * p.ld_out;
    const TT* __restrict__ taps = static_cast<const TT*>(p.taps_pm);
    const int K = p.K, D = p.D, tpp = p.tpp;
    const int nchunk = tpp / R;

    constexpr long NT = (long)kBlock * R;
    const long m0 = (long)blockIdx.x * NT;
    const int tid = threadIdx.x;

    if (m0 < p.n_out) {
        // LDS sample s <-> stream index gstart + s.  F = backward reach of the padded
        // polyphase windows (>= K-1), so every window read lands at s >= 0.
        const long F = (long)nchunk * R * D + D - 1;
        const long gstart = p.i0 + m0 * D - F;
        const long cnt = min(NT, p.n_out - m0);
        const long S = F + (cnt - 1) * D + 1;
        for (long s = tid; s < S; s += kBlock)
            lds[lds_index(s)] = fetch_stream(in, p.n_in, hist, K, gstart + s);
        __syncthreads();

        TS acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = zero_of<TS>();

        for (int ph = 0; ph < D; ++ph) {
            const TT* __restrict__ hp = taps + (long)ph * tpp;
            // window w[j] = lds sample (sbase + j*D); output r, tap i reads w[r - i].
            const long sbase = F - ph + (long)tid * R * D;
            TS cur[R], prev[R];
#pragma unroll
            for (int r = 0; r < R; ++r) cur[r] = lds[lds_index(sbase + (long)r * D)];
            for (int c = 0; c < nchunk; ++c) {
                const long pb = sbase - (long)(c + 1) * R * D;
#pragma unroll
                for (int q = 0; q < R; ++q) prev[q] = lds[lds_index(pb + (long)q * D)];
#pragma unroll
                for (int ii = 0; ii < R; ++ii) {
                    const TT h = hp[c * R + ii];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int pos = r - ii + R;  // index into [prev | cur]
                        mac(acc[r], pos < R ? prev[pos] : cur[pos - R], h);
                    }
                }
#pragma unroll
                for (int q = 0; q < R; ++q) cur[q] = prev[q];
            }
        }
        const long mq = m0 + (long)tid * R;
#pragma unroll
        for (int r = 0; r < R; ++r)  // non-finite outputs: the reference's sum (fir_exact.hpp)
            if (mq + r < p.n_out) out[mq + r] = fir_checked<TS, TT>(p, in, hist, mq + r, acc[r]);
    }

    if (blockIdx.x == gridDim.x - 1) {
        carry_history(in, p.n_in, hist,
                      static_cast<TS*>(p.hist_next) + ch * (long)(p.K - 1), K);
    }
}

// Fallback for shapes whose LDS tile would not fit (very large D*K): one lane per output,
// reads straight from HBM/L2.  Same taps layout.
template <typename TS, typename TT>
__global__ __launch_bounds__(kBlock) void fir_naive_kernel(FirParams p) {
    const long ch = blockIdx.y;
    const TS* __restrict__ in = static_cast<const TS*>(p.in) + ch * p.ld_in;
    const TS* __restrict__ hist = static_cast<const TS*>(p.hist) + ch * (long)(p.K - 1);
    TS* __restrict__ out = static_cast<TS*>(p.out) + ch * p.ld_out;
    const TT* __restrict__ taps = static_cast<const TT*>(p.taps_pm);
    const long m = (long)blockIdx.x * kBlock + threadIdx.x;
    if (m < p.n_out) {
        const long g = p.i0 + m * p.D;
        TS acc = zero_of<TS>();
        for (int k = 0; k < p.K; ++k) {
            const TT h = taps[(long)(k % p.D) * p.tpp + k / p.D];
            mac(acc, fetch_stream(in, p.n_in, hist, p.K, g - k), h);
        }
        out[m] = acc;
    }
    if (blockIdx.x == gridDim.x - 1) {
        carry_history(in, p.n_in, hist,
                      static_cast<TS*>(p.hist_next) + ch * (long)(p.K - 1), p.K);
    }
}

template <typename TS, typename TT, int R>
int launch_direct(const FirParams& p, hipStream_t s) {
    constexpr long NT = (long)kBlock * R;
    const long nchunk = p.tpp / R;
    const long F = nchunk * R * p.D + p.D - 1;
    const long S = F + (NT - 1) * p.D + 1;
    const size_t lds_bytes = (size_t)(lds_index(S) + 1) * sizeof(TS);
    const long nblk = p.n_out > 0 ? ceil_div(p.n_out, NT) : 1;
    dim3 grid((unsigned)nblk, (unsigned)p.nch);
    hipLaunchKernelGGL((fir_direct_kernel<TS, TT, R>), grid, dim3(kBlock), lds_bytes, s, p);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

template <typename TS, typename TT>
int launch_naive(const FirParams& p, hipStream_t s) {
    const long nblk = p.n_out > 0 ? ceil_div(p.n_out, kBlock) : 1;
    dim3 grid((unsigned)nblk, (unsigned)p.nch);
    hipLaunchKernelGGL((fir_naive_kernel<TS, TT>), grid, dim3(kBlock), 0, s, p);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

template <typename TS, typename TT>
int dispatch_direct(const FirParams& p, hipStream_t s) {
    // LDS budget per workgroup: keep <= 80 KiB so two workgroups share a CU.
    auto lds_for = [&](long R) {
        const long nchunk = p.tpp / R;
        const long F = nchunk * R * p.D + p.D - 1;
        const long S = F + ((long)kBlock * R - 1) * p.D + 1;
        return (lds_index(S) + 1) * (long)sizeof(TS);
    };
    constexpr long kBudget = 80 * 1024;
    if (p.force_naive) return launch_naive<TS, TT>(p, s);
    if (lds_for(8) <= kBudget) return launch_direct<TS, TT, 8>(p, s);
    if (lds_for(2) <= kBudget) return launch_direct<TS, TT, 2>(p, s);
    return launch_naive<TS, TT>(p, s);
}

}  // namespace

int fir_direct_launch(const FirParams& p, hipStream_t s) {
    if (!p.force_naive && fir_direct2_supported(p)) return fir_direct2_launch(p, s);
    if (p.sample_kind == SDRGPU_F32 && p.tap_kind == SDRGPU_F32)
        return dispatch_direct<float, float>(p, s);
    if (p.sample_kind == SDRGPU_C64 && p.tap_kind == SDRGPU_F32)
        return dispatch_direct<c64, float>(p, s);
    if (p.sample_kind == SDRGPU_C64 && p.tap_kind == SDRGPU_C64)
        return dispatch_direct<c64, c64>(p, s);
    return SDRGPU_ERR_INVALID;
}

}  // namespace sdrgpu
