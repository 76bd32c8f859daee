// biquad_kernels.hpp -- device-side entry points of biquad.hip (batched Biquad<C, f32>).
#pragma once

#include <hip/hip_runtime.h>

namespace sdrgpu {

// DF1 state of one channel (biquad.rs:4-22): inputs x1, x2 and outputs y1, y2; re / im for
// Complex<f32> samples (the im fields stay 0 for f32 samples)
struct BiquadState {
    float x1r, x1i, x2r, x2i, y1r, y1i, y2r, y2i;
};

// time-parallel plan and scratch of one block (abi_biquad.cpp; the bq_*_kernel of biquad.hip)
struct BqSpec {
    long seg = 0, warm = 0, ck = 0, nseg = 0;
    BiquadState *guess = nullptr, *end = nullptr, *end2 = nullptr, *ckpt = nullptr;
    int* rstop = nullptr;
    unsigned long long* recomputed = nullptr;  // segments whose guess missed (zeroed per block)
};

// one serial pass per channel (one lane each)
int biquad_launch(bool cplx, long nch, const float* c, int ident, const void* in, long ld_in,
                  long n, void* out, long ld_out, BiquadState* state, hipStream_t s);
// time-parallel: segments of sp.seg samples per channel, warm-up sp.warm, checkpoints sp.ck
int biquad_tp_launch(bool cplx, long nch, const float* c, const void* in, long ld_in, long n,
                     void* out, long ld_out, BiquadState* state, const BqSpec& sp, hipStream_t s);

}  // namespace sdrgpu
