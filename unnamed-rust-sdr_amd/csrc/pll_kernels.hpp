// pll_kernels.hpp -- internal launch interface of the batched PLL kernel.
#pragma once

#include "common.hpp"

namespace sdrgpu {

struct PllDevParams {
    long nch;
    float rate;       // Pll::rate (pll.rs:50)
    float reference;  // reference / rate (pll.rs:51)
    float gain;       // pll.rs:52
    float loopc[5], outc[5], lockc[5];  // b0 b1 b2 na1 na2 (biquad.rs:25-38)
    int loop_ident, out_ident, lock_ident;
    int out_mode;     // SDRGPU_PLL_OUT_FILTER (0) or SDRGPU_PLL_OUT_STEREO_DIFF (1)
    int in_u8;        // input = rtl_tcp interleaved u8 I/Q (2 B/sample), (v - 128) / 128
};

// Per-channel state (Pll fields nphase/value + three biquad states), 20 floats.
struct PllChannelState {
    float nphase, vr, vi;
    float lx1r, lx1i, lx2r, lx2i, ly1r, ly1i, ly2r, ly2i;  // loop filter (complex)
    float ox1, ox2, oy1, oy2;                               // output filter
    float kx1, kx2, ky1, ky2;                               // lock filter
    float pad;
};

// Time-parallel plan of one block (pll.hip, "speculative segments"): seg > 0 cuts each
// channel's n samples into ceil(n / seg) segments run concurrently, each after `warm` samples
// of warm-up from the design state; guess / end hold [segments][nch] states (the state each
// segment's warm-up reached at its start, and the state at its end).  seg == 0: one serial pass.
struct PllSpec {
    long seg = 0, warm = 0;
    PllChannelState* guess = nullptr;
    PllChannelState* end = nullptr;
    unsigned long long* recomputed = nullptr;  // segments pll_fix_kernel ran again (zeroed per block)
    long ck = 0;                               // checkpoint interval inside a segment
    PllChannelState* ckpt = nullptr;           // [segments][nch][seg / ck - 1] states at t0 + j ck
    // parallel re-run (pll_refix_kernel): per segment, +k = re-run from the previous segment's
    // end met this trajectory after k intervals, -k = ran k intervals without meeting it (end
    // state in end2), 0 = not re-run
    int* rstop = nullptr;
    PllChannelState* end2 = nullptr;
    // optional: four events recorded around pass 1, the re-run pass and the walk
    hipEvent_t* phase_ev = nullptr;
};

int pll_launch(const PllDevParams& p, const void* in, long ld_in, long n, float* out,
               uint8_t* locked, long ld_out, PllChannelState* state, const PllSpec& spec,
               hipStream_t s);

// test-only: the device atan2f (fn 0) / sincosf (fn 1) restatements over n operands
int libm_debug_launch(int fn, const float* a, const float* b, float* o0, float* o1, long n,
                      hipStream_t s);

}  // namespace sdrgpu
