// common.hpp -- shared device/host helpers for the sdrgpu HIP core (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/sdrgpu.h"

namespace sdrgpu {

// Complex sample as stored in HBM: num::Complex<f32> layout (#[repr(C)] {re, im}).
using c64 = float2;

// -------- MAC primitive: Convolve::accumulate (src/filter/convolve.rs:13-15) --------
// acc += x * h with the num-complex product; fused (FMA) on the GPU, which is the only
// numeric difference from the reference (tolerance 1e-5 of RMS).
__device__ __forceinline__ void mac(float& acc, float x, float h) { acc = fmaf(x, h, acc); }
__device__ __forceinline__ void mac(c64& acc, c64 x, float h) {
    acc.x = fmaf(x.x, h, acc.x);
    acc.y = fmaf(x.y, h, acc.y);
}
__device__ __forceinline__ void mac(c64& acc, c64 x, c64 h) {
    acc.x = fmaf(x.x, h.x, acc.x);
    acc.x = fmaf(-x.y, h.y, acc.x);
    acc.y = fmaf(x.x, h.y, acc.y);
    acc.y = fmaf(x.y, h.x, acc.y);
}

template <typename T> __device__ __forceinline__ T zero_of();
template <> __device__ __forceinline__ float zero_of<float>() { return 0.0f; }
template <> __device__ __forceinline__ c64 zero_of<c64>() { return make_float2(0.0f, 0.0f); }

__host__ __device__ constexpr inline long ceil_div(long a, long b) { return (a + b - 1) / b; }

// -------- SIMD ownership --------
// No wave of another kernel may share a SIMD with MFMA FIR waves: a packed-f32 VALU result was
// read wrongly (lanes 48-63) by a PLL wave co-resident with MFMA bank waves.
// A wave's register claim decides what else fits on its SIMD, so both sides claim the file:
// the MFMA FIR kernels run two waves per SIMD and each names v255 (2 x 256 = 512 VGPRs, no
// AGPRs), the one-wave-per-SIMD kernels (PLL, biquad, the bf16x3 FIR) name v255 and a255.
// Only the kernel's VGPR count changes (the instruction stream is the same; checked by
// tests/test_kernel_resources_cpu.py on the shipped code object).
__device__ __forceinline__ void claim_simd_half() { asm volatile("" ::: "v255"); }
__device__ __forceinline__ void claim_simd_whole() { asm volatile("" ::: "v255", "a255"); }

}  // namespace sdrgpu

// Host-side error plumbing shared by the ABI translation units.
#define SDRGPU_HIP_TRY(expr)                                   \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) {                                \
            sdrgpu::detail::set_last_hip_error(e_);            \
            return (e_ == hipErrorOutOfMemory ||               \
                    e_ == hipErrorMemoryAllocation)            \
                       ? SDRGPU_ERR_NOMEM                      \
                       : SDRGPU_ERR_DEVICE;                    \
        }                                                      \
    } while (0)

#define SDRGPU_LAUNCH_CHECK()                                  \
    do {                                                       \
        hipError_t e_ = hipGetLastError();                     \
        if (e_ != hipSuccess) {                                \
            sdrgpu::detail::set_last_hip_error(e_);            \
            return SDRGPU_ERR_LAUNCH;                          \
        }                                                      \
    } while (0)

namespace sdrgpu {
namespace detail {
void set_last_hip_error(hipError_t e);
}
}  // namespace sdrgpu
