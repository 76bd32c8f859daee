// fdiv_check.hip -- GPU check that sdr_fdiv (libm_glibc.h: f64 reciprocal + Newton +
// corrected quotient, rounded once to f32) is bit-identical to the compiler's IEEE a / b for
// every finite nonzero pair whose quotient is a normal float: 2^36 hashed random pairs (all
// mantissas and signs, exponents over the whole range incl. subnormal operands) plus pairs
// whose quotient sits next to a rounding boundary (a = fl(b * q) nudged by one ulp).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++20 fdiv_check.hip -o fdiv_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return (uint32_t)x;
}
__device__ __forceinline__ float in_window(uint32_t h) {  // exponent 0..254 (subnormals too)
    const uint32_t e = (h >> 23) % 255u;
    return __uint_as_float((h & 0x807fffffu) | (e << 23));
}
#include "../unnamed-rust-sdr_amd/csrc/libm_glibc.h"
__device__ __forceinline__ float fast_div(float a, float b) { return sdr_fdiv(a, b); }
__global__ void check(uint64_t base, unsigned long long* bad, uint32_t* ex) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float a, b;
    if (i & 1) {
        a = in_window(mix(2 * i));
        b = in_window(mix(2 * i + 1));
    } else {  // near-boundary quotients: a = fl(b * q) nudged by +-1 ulp
        b = in_window(mix(2 * i + 1));
        float q = in_window(mix(2 * i));
        const uint32_t qe = (__float_as_uint(q) >> 23) & 0xff;
        if (qe > 127 + 60 || qe < 127 - 60) q = __uint_as_float((__float_as_uint(q) & 0x807fffffu) | (127u << 23));
        a = b * q;
        const int nud = (int)(mix(3 * i) % 3) - 1;
        a = __uint_as_float(__float_as_uint(a) + nud);
    }
    const float x = a / b;
    const uint32_t xe = (__float_as_uint(x) >> 23) & 0xff;
    if (a == 0.f || b == 0.f || xe == 0 || xe == 255 || ((__float_as_uint(a) >> 23) & 0xff) == 255) return;
    const float y = fast_div(a, b);
    if (__float_as_uint(x) != __float_as_uint(y)) {
        const unsigned long long k = atomicAdd(bad, 1ULL);
        if (k < 4) {
            ex[4 * k] = __float_as_uint(a); ex[4 * k + 1] = __float_as_uint(b);
            ex[4 * k + 2] = __float_as_uint(x); ex[4 * k + 3] = __float_as_uint(y);
        }
    }
}
int main() {
    unsigned long long* bad;
    uint32_t* ex;
    hipMalloc(&bad, 8);
    hipMalloc(&ex, 64);
    hipMemset(bad, 0, 8);
    const uint64_t per = 1ULL << 30;
    for (uint64_t b = 0; b < (1ULL << 36); b += per) {
        hipLaunchKernelGGL(check, dim3((unsigned)(per / 256)), dim3(256), 0, 0, b, bad, ex);
        if (((b / per) & 7) == 7) { hipDeviceSynchronize(); printf("checked %llu\n", (unsigned long long)(b + per)); fflush(stdout); }
    }
    unsigned long long nb = 0;
    uint32_t h[16] = {};
    hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(h, ex, 64, hipMemcpyDeviceToHost);
    printf("pairs 2^36, mismatches %llu\n", nb);
    for (unsigned k = 0; k < (nb < 4 ? nb : 4); ++k)
        printf("  a=%08x b=%08x div=%08x fast=%08x\n", h[4 * k], h[4 * k + 1], h[4 * k + 2], h[4 * k + 3]);
    return nb ? 1 : 0;
}
