// atanf_check.hip -- GPU check that sdr_atanf_bf (libm_glibc.h, whose argument reduction divides
// with sdr_fdiv_n: f32 reciprocal + Newton + two corrected quotients, no operand scaling) is
// bit-identical to the same function dividing with the IEEE operator, for EVERY non-negative
// finite float argument (bit patterns 0 .. 0x7f7fffff) -- the whole domain atan2f's common
// path calls it on (|y / x|).  The host C build of libm_glibc.h divides with '/', and
// tests/libm_check.c checks that against this machine's glibc.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++20 atanf_check.hip -o atanf_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../unnamed-rust-sdr_amd/csrc/libm_glibc.h"

__global__ void check(uint32_t base, unsigned long long* bad, uint32_t* ex) {
    const uint32_t i = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 0x7f800000u) return;
    const float x = __uint_as_float(i);
    const float a = sdr_atanf_core(x, 1);
    const float b = sdr_atanf_bf(x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
        const unsigned long long k = atomicAdd(bad, 1ULL);
        if (k < 4) {
            ex[3 * k] = i; ex[3 * k + 1] = __float_as_uint(a); ex[3 * k + 2] = __float_as_uint(b);
        }
    }
}
int main() {
    unsigned long long* bad;
    uint32_t* ex;
    hipMalloc(&bad, 8);
    hipMalloc(&ex, 64);
    hipMemset(bad, 0, 8);
    const uint32_t per = 1u << 26;
    for (uint32_t b = 0; b < 0x7f800000u; b += per)
        hipLaunchKernelGGL(check, dim3(per / 256), dim3(256), 0, 0, b, bad, ex);
    hipDeviceSynchronize();
    unsigned long long nb = 0;
    uint32_t h[12] = {};
    hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(h, ex, 48, hipMemcpyDeviceToHost);
    printf("atanf arguments 0 .. 0x7f7fffff (%u), mismatches %llu\n", 0x7f800000u, nb);
    for (unsigned k = 0; k < (nb < 4 ? nb : 4); ++k)
        printf("  x=%08x ieee=%08x fast=%08x\n", h[3 * k], h[3 * k + 1], h[3 * k + 2]);
    return nb ? 1 : 0;
}
