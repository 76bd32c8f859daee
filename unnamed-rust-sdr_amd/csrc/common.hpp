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
