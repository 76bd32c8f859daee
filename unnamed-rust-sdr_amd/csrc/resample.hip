// resample.hip -- sample arithmetic of libsamplerate's zero-order-hold and linear converters
// (the src_zoh.c / src_linear.c process loops behind SampleRate::process, reference
// src/resample.rs:46-67).  The host walks the data-independent f64 position recurrence
// (abi_resample.cpp) and hands each output frame k its left source frame L[k] (-1 = the
// carried last_value) and, for linear, the fraction f[k]; this kernel evaluates
//     ZOH:    out = x[L]
//     linear: out = (float)((double)x[L] + f * ((double)x[L+1] - (double)x[L]))
// for every (frame, channel), in the converter's f64 operation order with explicit
// round-to-nearest ops (no contraction), so outputs are bit-identical to libsamplerate's.
// Frames are channel-interleaved, so consecutive lanes read consecutive channels of the
// same frame: for a batch of many streams (large `channels`) every load is coalesced and
// the L / f table is a per-frame broadcast.  HBM bound: 4 B in (+ neighbour reuse from L2)
// + 4 B out per sample.
#include "common.hpp"
#include "resample_kernels.hpp"

namespace sdrgpu {

namespace {

constexpr int kSrcBlock = 256;
constexpr int kSrcRows = 4;  // frames per workgroup in the wide-frame kernel

template <bool LINEAR>
__device__ __forceinline__ float src_eval(const float* __restrict__ in, long channels, int l,
                                          double f, long ch, const float* __restrict__ lv) {
    const float a = l < 0 ? lv[ch] : in[(long)l * channels + ch];
    if constexpr (LINEAR) {
        const float b = in[((long)l + 1) * channels + ch];
        const double da = (double)a;
        return (float)__dadd_rn(da, __dmul_rn(f, __dsub_rn((double)b, da)));
    } else {
        return a;
    }
}

// Wide frames (channels >= 64, e.g. a batch of streams): blockIdx.x = a run of kSrcRows
// output frames, blockIdx.y tiles the channels of a frame; the (left, frac) of a frame is
// uniform across the workgroup (scalar loads), every sample load / store is coalesced.
template <bool LINEAR>
__global__ __launch_bounds__(kSrcBlock) void src_interp_wide_kernel(
    const float* __restrict__ in, long channels, const int* __restrict__ left,
    const double* __restrict__ frac, long nframes, const float* __restrict__ last_value,
    float* __restrict__ out) {
    const long ch = (long)blockIdx.y * kSrcBlock + threadIdx.x;
    const long k0 = (long)blockIdx.x * kSrcRows;
    if (ch >= channels) return;
#pragma unroll
    for (int r = 0; r < kSrcRows; ++r) {
        const long k = k0 + r;
        if (k >= nframes) break;
        out[k * channels + ch] =
            src_eval<LINEAR>(in, channels, left[k], LINEAR ? frac[k] : 0.0, ch, last_value);
    }
}

// Narrow frames (1..63 channels): one sample per lane over the flattened (frame, channel)
// index; CH > 0 fixes the channel count at compile time (1 = f32, 2 = Complex<f32>).
template <bool LINEAR, int CH>
__global__ __launch_bounds__(kSrcBlock) void src_interp_kernel(
    const float* __restrict__ in, long channels, const int* __restrict__ left,
    const double* __restrict__ frac, long nframes, const float* __restrict__ last_value,
    float* __restrict__ out) {
    const long C = CH > 0 ? CH : channels;
    const long total = nframes * C;
    const long stride = (long)gridDim.x * kSrcBlock;
    for (long t = (long)blockIdx.x * kSrcBlock + threadIdx.x; t < total; t += stride) {
        const long k = CH > 0 ? t / CH : (long)((unsigned long)t / (unsigned long)C);
        const long ch = t - k * C;
        out[t] = src_eval<LINEAR>(in, C, left[k], LINEAR ? frac[k] : 0.0, ch, last_value);
    }
}

template <bool LINEAR>
void src_launch_t(const float* in, long channels, const int* left, const double* frac,
                  long nframes, const float* lv, float* out, hipStream_t s) {
    if (channels >= 64) {
        const dim3 grid((unsigned)((nframes + kSrcRows - 1) / kSrcRows),
                        (unsigned)((channels + kSrcBlock - 1) / kSrcBlock));
        src_interp_wide_kernel<LINEAR><<<grid, kSrcBlock, 0, s>>>(in, channels, left, frac,
                                                                  nframes, lv, out);
        return;
    }
    long blocks = (nframes * channels + kSrcBlock - 1) / kSrcBlock;
    if (blocks > 65536) blocks = 65536;
    const unsigned g = (unsigned)blocks;
    if (channels == 1)
        src_interp_kernel<LINEAR, 1><<<g, kSrcBlock, 0, s>>>(in, 1, left, frac, nframes, lv, out);
    else if (channels == 2)
        src_interp_kernel<LINEAR, 2><<<g, kSrcBlock, 0, s>>>(in, 2, left, frac, nframes, lv, out);
    else
        src_interp_kernel<LINEAR, 0><<<g, kSrcBlock, 0, s>>>(in, channels, left, frac, nframes,
                                                             lv, out);
}

}  // namespace

int src_interp_launch(bool linear, const float* in, long channels, const int* left,
                      const double* frac, long nframes, const float* last_value, float* out,
                      hipStream_t s) {
    if (nframes <= 0 || channels <= 0) return SDRGPU_OK;
    if ((nframes + kSrcRows - 1) / kSrcRows > 0x7fffffffL ||
        (channels + kSrcBlock - 1) / kSrcBlock > 65535)
        return SDRGPU_ERR_UNSUPPORTED;
    if (linear)
        src_launch_t<true>(in, channels, left, frac, nframes, last_value, out, s);
    else
        src_launch_t<false>(in, channels, left, frac, nframes, last_value, out, s);
    return hipGetLastError() == hipSuccess ? SDRGPU_OK : SDRGPU_ERR_LAUNCH;
}


// ---- sinc converters (libsamplerate src_sinc.c calc_output_multi) ----------------------
// The host (abi_resample.cpp) restates src_sinc.c's buffer bookkeeping (prepare_data, the
// fixed-point filter index, the ratio ramp, termination) over integers only and hands each
// output frame a descriptor: where its left half starts (window sample index + filter
// index, after libsamplerate's underflow skip), where its right half starts, the tap
// counts, the fixed-point increment and the output scale.  This kernel evaluates
//     left  = sum over the left taps  (data index ascending)  of icoeff * x
//     right = sum over the right taps (data index descending) of icoeff * x
//     icoeff = c[i] + frac * (c[i+1] - c[i])   (f32 difference, f64 product and sum)
//     out   = (float)(scale * (left + right))
// in that f64 order with explicit round-to-nearest ops, one (frame, channel) per lane, so
// outputs are bit-identical to the restatement.  The window holds the stream samples the
// libsamplerate buffer would hold (channel-interleaved), so lanes of one frame read
// consecutive channels.  Per output ~2 * half_len / increment taps (SincFastest at ratio
// 0.08: ~480): FP64-issue bound, not HBM bound.


namespace {

__device__ __forceinline__ double sinc_icoeff(const float* __restrict__ c, int fi) {
    const double frac = (double)(fi & 4095) * (1.0 / 4096.0);
    const int i = fi >> 12;
    const float c0 = c[i], c1 = c[i + 1];
    return __dadd_rn((double)c0, __dmul_rn(frac, (double)__fsub_rn(c1, c0)));
}

template <int CH>
__global__ __launch_bounds__(kSrcBlock) void src_sinc_kernel(
    const float* __restrict__ win, long channels, const SincDesc* __restrict__ desc,
    long nframes, const float* __restrict__ coeffs, float* __restrict__ out) {
    const long C = CH > 0 ? CH : channels;
    const long total = nframes * C;
    const long stride = (long)gridDim.x * kSrcBlock;
    for (long t = (long)blockIdx.x * kSrcBlock + threadIdx.x; t < total; t += stride) {
        const long k = CH > 0 ? t / CH : (long)((unsigned long)t / (unsigned long)C);
        const long ch = t - k * C;
        const SincDesc d = desc[k];
        double left = 0.0, right = 0.0;
        int fi = d.fil;
        long x = (long)d.dl + ch;
        for (int n = 0; n < d.nl; ++n) {
            left = __dadd_rn(left, __dmul_rn(sinc_icoeff(coeffs, fi), (double)win[x]));
            fi -= d.inc;
            x += C;
        }
        fi = d.fir;
        x = (long)d.dr + ch;
        for (int n = 0; n < d.nr; ++n) {
            right = __dadd_rn(right, __dmul_rn(sinc_icoeff(coeffs, fi), (double)win[x]));
            fi -= d.inc;
            x -= C;
        }
        out[t] = (float)__dmul_rn(d.scale, __dadd_rn(left, right));
    }
}

// Wide frames (channels >= 64, a batch of streams sharing one ratio): a workgroup takes one
// output frame x 256 channels.  The frame's descriptor is uniform, so its interpolated
// coefficients are computed once per workgroup into LDS (in chunks of kTapChunk taps) and
// every lane reads them as broadcasts; the tap sums stay sequential per lane (same order,
// same roundings as the narrow kernel).  Workgroups b, b+8, b+16, ... share an XCD (round-
// robin placement, speed only): each XCD gets a contiguous range of frames, so the window
// samples that neighbouring frames share are read from HBM once into that XCD's L2.
constexpr int kTapChunk = 1024;

__global__ __launch_bounds__(kSrcBlock) void src_sinc_wide_kernel(
    const float* __restrict__ win, long channels, const SincDesc* __restrict__ desc,
    long nframes, const float* __restrict__ coeffs, float* __restrict__ out, int ntiles,
    long per_xcd) {
    __shared__ double ic[kTapChunk];
    const long b = blockIdx.x;
    const long logical = (b & 7) * per_xcd + (b >> 3);
    if (logical >= nframes * ntiles) return;  // whole workgroup: no barrier is skipped
    const long k = logical / ntiles;
    const long ch = (logical - k * ntiles) * kSrcBlock + threadIdx.x;
    const bool on = ch < channels;
    const SincDesc d = desc[k];
    double acc[2] = {0.0, 0.0};
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        const int n = side ? d.nr : d.nl, fi0 = side ? d.fir : d.fil;
        const long step = side ? -channels : channels;
        long x = (long)(side ? d.dr : d.dl) + ch;
        double a = 0.0;
        for (int base = 0; base < n; base += kTapChunk) {
            const int m = n - base < kTapChunk ? n - base : kTapChunk;
            for (int j = threadIdx.x; j < m; j += kSrcBlock)
                ic[j] = sinc_icoeff(coeffs, fi0 - (base + j) * d.inc);
            __syncthreads();
            if (on) {
#pragma unroll 4
                for (int j = 0; j < m; ++j) {
                    a = __dadd_rn(a, __dmul_rn(ic[j], (double)win[x]));
                    x += step;
                }
            }
            __syncthreads();
        }
        acc[side] = a;
    }
    if (on) out[k * channels + ch] = (float)__dmul_rn(d.scale, __dadd_rn(acc[0], acc[1]));
}

}  // namespace

int src_sinc_launch(const float* win, long channels, const SincDesc* desc, long nframes,
                    const float* coeffs, float* out, hipStream_t s) {
    if (nframes <= 0 || channels <= 0) return SDRGPU_OK;
    if (channels >= 64) {
        const int ntiles = (int)((channels + kSrcBlock - 1) / kSrcBlock);
        const long per_xcd = (nframes * ntiles + 7) / 8;
        if (8 * per_xcd > 0x7fffffffL) return SDRGPU_ERR_UNSUPPORTED;
        src_sinc_wide_kernel<<<(unsigned)(8 * per_xcd), kSrcBlock, 0, s>>>(
            win, channels, desc, nframes, coeffs, out, ntiles, per_xcd);
        return hipGetLastError() == hipSuccess ? SDRGPU_OK : SDRGPU_ERR_LAUNCH;
    }
    long blocks = (nframes * channels + kSrcBlock - 1) / kSrcBlock;
    if (blocks > 65536) blocks = 65536;
    const unsigned g = (unsigned)blocks;
    if (channels == 1)
        src_sinc_kernel<1><<<g, kSrcBlock, 0, s>>>(win, 1, desc, nframes, coeffs, out);
    else if (channels == 2)
        src_sinc_kernel<2><<<g, kSrcBlock, 0, s>>>(win, 2, desc, nframes, coeffs, out);
    else
        src_sinc_kernel<0><<<g, kSrcBlock, 0, s>>>(win, channels, desc, nframes, coeffs, out);
    return hipGetLastError() == hipSuccess ? SDRGPU_OK : SDRGPU_ERR_LAUNCH;
}

}  // namespace sdrgpu
