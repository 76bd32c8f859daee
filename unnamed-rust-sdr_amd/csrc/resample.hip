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

// Mono / stereo streams (src/main.rs:50 resamples the mono FM audio with SincFastest): one
// lane per output frame leaves each lane a serial chain of ~481 taps, each waiting on its
// loads (59 us for a 4096-sample call, 2 workgroups on the whole chip).  The products do not
// depend on the running sums, only the sums are ordered, so a workgroup takes kSincItems
// (frame, channel) items: its 256 lanes first compute every tap product of the items in
// parallel (window span and, when short, the coefficient table staged in LDS) into an f64
// LDS array, then one lane per item adds its products in the reference order (left taps
// ascending, right taps descending: the same __dmul_rn / __dadd_rn values and order as the
// global path, so outputs are bit-identical).  Items whose products do not fit take the
// sequential path below.
constexpr int kSincItems = 8;
constexpr int kProdLds = 8192;   // f64 products per workgroup (64 KiB): 8 items of <= 1024 taps
constexpr int kWinLds = 4096;    // window floats staged per workgroup (16 KiB)
constexpr int kCoefLds = 4096;   // coefficient floats staged when the table fits (16 KiB)

template <int CH>
__global__ __launch_bounds__(kSrcBlock) void src_sinc_lds_kernel(
    const float* __restrict__ win, const SincDesc* __restrict__ desc, long nframes,
    const float* __restrict__ coeffs, int coeff_len, float* __restrict__ out) {
    __shared__ double prod[kProdLds];
    __shared__ float wl[kWinLds];
    __shared__ float cl[kCoefLds];
    __shared__ int pofs[kSincItems + 1];
    __shared__ SincDesc sd[kSincItems];
    __shared__ long span_lo, span_hi;
    constexpr long C = CH;
    const long total = nframes * C;
    const long t0 = (long)blockIdx.x * kSincItems;
    const int ni = (int)(total - t0 < kSincItems ? total - t0 : kSincItems);
    if (threadIdx.x < 64) {  // wave 0: the items' descriptors (one load per lane, in parallel),
                             // product offsets (prefix sum) and the window span
        const int i = threadIdx.x;
        long lo = 0x7fffffffffffL, hi = -0x7fffffffffffL;
        int cnt = 0;
        if (i < ni) {
            const long t = t0 + i, k = t / CH, ch = t - k * CH;
            const SincDesc d = desc[k];
            sd[i] = d;
            cnt = (d.nl > 0 ? d.nl : 0) + d.nr;
            if (d.nl > 0) {
                lo = min(lo, (long)d.dl + ch);
                hi = max(hi, (long)d.dl + ch + (long)(d.nl - 1) * C);
            }
            lo = min(lo, (long)d.dr + ch - (long)(d.nr - 1) * C);
            hi = max(hi, (long)d.dr + ch);
        }
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < kSincItems; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (i >= o) incl += v;
        }
#pragma unroll
        for (int o = kSincItems / 2; o > 0; o >>= 1) {
            lo = min(lo, (long)__shfl_xor(lo, o));
            hi = max(hi, (long)__shfl_xor(hi, o));
        }
        if (i < kSincItems) pofs[i + 1] = incl;
        if (i == 0) {
            pofs[0] = 0;
            span_lo = lo;
            span_hi = hi;
        }
    }
    __syncthreads();
    const int np = pofs[ni];
    const long base = span_lo, n = span_hi - span_lo + 1;
    const bool fits = np <= kProdLds && n > 0 && n <= kWinLds;  // workgroup-uniform
    if (!fits) {  // sequential path (very long filters / extreme ratios)
        if (threadIdx.x < ni) {
            const long t = t0 + threadIdx.x, k = t / CH, ch = t - k * CH;
            const SincDesc d = desc[k];
            double left = 0.0, right = 0.0;
            int fi = d.fil;
            long x = (long)d.dl + ch;
            for (int m = 0; m < d.nl; ++m) {
                left = __dadd_rn(left, __dmul_rn(sinc_icoeff(coeffs, fi), (double)win[x]));
                fi -= d.inc;
                x += C;
            }
            fi = d.fir;
            x = (long)d.dr + ch;
            for (int m = 0; m < d.nr; ++m) {
                right = __dadd_rn(right, __dmul_rn(sinc_icoeff(coeffs, fi), (double)win[x]));
                fi -= d.inc;
                x -= C;
            }
            out[t] = (float)__dmul_rn(d.scale, __dadd_rn(left, right));
        }
        return;
    }
    const bool lds_coef = coeff_len <= kCoefLds;
    for (int i = threadIdx.x; i < (int)n; i += kSrcBlock) wl[i] = win[base + i];
    if (lds_coef)
        for (int i = threadIdx.x; i < coeff_len; i += kSrcBlock) cl[i] = coeffs[i];
    __syncthreads();
    const float* cs = lds_coef ? cl : coeffs;
    // phase 1: every product of the block's items, in parallel
    for (int g = threadIdx.x; g < np; g += kSrcBlock) {
        int i = 0;
        while (i + 1 < ni && pofs[i + 1] <= g) ++i;
        const long t = t0 + i, k = t / CH, ch = t - k * CH;
        const SincDesc& d = sd[i];
        const int m = g - pofs[i], nl = d.nl > 0 ? d.nl : 0;
        int fi;
        long x;
        if (m < nl) {
            fi = d.fil - m * d.inc;
            x = (long)d.dl + ch + (long)m * C;
        } else {
            fi = d.fir - (m - nl) * d.inc;
            x = (long)d.dr + ch - (long)(m - nl) * C;
        }
        prod[g] = __dmul_rn(sinc_icoeff(cs, fi), (double)wl[x - base]);
    }
    __syncthreads();
    // phase 2: one lane per item sums its products in the reference order
    if (threadIdx.x < ni) {
        const int i = threadIdx.x;
        const long t = t0 + i;
        const SincDesc& d = sd[i];
        const int nl = d.nl > 0 ? d.nl : 0, o = pofs[i];
        double left = 0.0, right = 0.0;
#pragma unroll 8
        for (int m = 0; m < nl; ++m) left = __dadd_rn(left, prod[o + m]);
#pragma unroll 8
        for (int m = 0; m < d.nr; ++m) right = __dadd_rn(right, prod[o + nl + m]);
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
                    const float* coeffs, int coeff_len, float* out, hipStream_t s) {
    if (nframes <= 0 || channels <= 0) return SDRGPU_OK;
    if ((channels == 1 || channels == 2) && (nframes * channels + kSincItems - 1) / kSincItems <= 0x7fffffffL) {
        const unsigned g = (unsigned)((nframes * channels + kSincItems - 1) / kSincItems);
        if (channels == 1)
            src_sinc_lds_kernel<1><<<g, kSrcBlock, 0, s>>>(win, desc, nframes, coeffs, coeff_len, out);
        else
            src_sinc_lds_kernel<2><<<g, kSrcBlock, 0, s>>>(win, desc, nframes, coeffs, coeff_len, out);
        return hipGetLastError() == hipSuccess ? SDRGPU_OK : SDRGPU_ERR_LAUNCH;
    }
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
