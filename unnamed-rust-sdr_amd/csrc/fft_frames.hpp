// fft_frames.hpp -- frame sources and output collation shared by the FFT kernels
// (power-of-two tiles / four-step in fft.hip, mixed-radix and Bluestein in fft_gen.hip).
#pragma once

#include "common.hpp"

namespace sdrgpu {

// -------- frame sources ---------------------------------------------------------------
struct FrameSrc {
    // mode 0: contiguous frames (frame f at in + f*M)
    // mode 1: STFT frames from a stream: frame f covers stream [f0 + (f+1)hop - M, +M), stream
    //         index g < 0 -> hist[g + H] (H = history length) if g >= -H, else 0; g >= n_in -> 0
    // mode 2: contiguous REAL frames (float, imag = 0) -- rfft
    int mode;
    const float2* in;
    const float* in_real;
    long n_in;
    const float2* hist;
    long H;
    long first_end;  // stream index (exclusive end) of frame 0 of this launch
    long hop;
};

__device__ __forceinline__ float2 frame_sample(const FrameSrc& s, long M, long f, long n) {
    if (s.mode == 0) return s.in[f * M + n];
    if (s.mode == 2) return make_float2(s.in_real[f * M + n], 0.f);
    const long g = s.first_end + f * s.hop - M + n;
    if (g >= 0) return g < s.n_in ? s.in[g] : make_float2(0.f, 0.f);
    if (g >= -s.H) return s.hist[g + s.H];
    return make_float2(0.f, 0.f);
}

// bin k of frame f by store mode: 0 collated fft (out[(k + M/2) mod M] * norm, fft.rs:14-26),
// 1 rfft (collated [M/2, M) = X[0, M - M/2) * norm, fft.rs:35), 2 natural order, unscaled
// (internal: the power-of-two transforms inside Bluestein)
__device__ __forceinline__ void store_bin(float2* __restrict__ out, long f, long M, long k,
                                          float2 x, int mode, float norm) {
    if (mode == 0) {
        long o = k + M / 2;
        if (o >= M) o -= M;
        out[f * M + o] = make_float2(x.x * norm, x.y * norm);
    } else if (mode == 1) {
        const long keep = M - M / 2;
        if (k < keep) out[f * keep + k] = make_float2(x.x * norm, x.y * norm);
    } else {
        out[f * M + k] = x;
    }
}


}  // namespace sdrgpu
