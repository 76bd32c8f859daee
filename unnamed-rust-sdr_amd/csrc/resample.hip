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

namespace sdrgpu {

namespace {

constexpr int kSrcBlock = 256;

template <bool LINEAR>
__global__ __launch_bounds__(kSrcBlock) void src_interp_kernel(
    const float* __restrict__ in, long channels, const int* __restrict__ left,
    const double* __restrict__ frac, long nframes, const float* __restrict__ last_value,
    float* __restrict__ out) {
    const long total = nframes * channels;
    const long stride = (long)gridDim.x * kSrcBlock;
    for (long t = (long)blockIdx.x * kSrcBlock + threadIdx.x; t < total; t += stride) {
        const long k = t / channels;
        const long ch = t - k * channels;
        const int l = left[k];
        const float a = l < 0 ? last_value[ch] : in[(long)l * channels + ch];
        if constexpr (LINEAR) {
            const float b = in[((long)l + 1) * channels + ch];
            const double da = (double)a;
            out[t] = (float)__dadd_rn(da, __dmul_rn(frac[k], __dsub_rn((double)b, da)));
        } else {
            out[t] = a;
        }
    }
}

}  // namespace

int src_interp_launch(bool linear, const float* in, long channels, const int* left,
                      const double* frac, long nframes, const float* last_value, float* out,
                      hipStream_t s) {
    const long total = nframes * channels;
    if (total <= 0) return SDRGPU_OK;
    long blocks = (total + kSrcBlock - 1) / kSrcBlock;
    if (blocks > 65536) blocks = 65536;
    if (linear)
        src_interp_kernel<true><<<(unsigned)blocks, kSrcBlock, 0, s>>>(in, channels, left, frac,
                                                                       nframes, last_value, out);
    else
        src_interp_kernel<false><<<(unsigned)blocks, kSrcBlock, 0, s>>>(in, channels, left, frac,
                                                                        nframes, last_value, out);
    return hipGetLastError() == hipSuccess ? SDRGPU_OK : SDRGPU_ERR_LAUNCH;
}

}  // namespace sdrgpu
