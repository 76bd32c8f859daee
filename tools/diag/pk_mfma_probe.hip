// pk_mfma_probe.hip -- round 5: is a packed-f32 result misread by the next dependent packed op
// when MFMA waves of another kernel share the SIMD?  (Diagnostic for DESIGN.md 3.6; not product.)
//
// victim:    one 64-lane wave per workgroup, 96 VGPRs, looping over the PLL mixer's exact pair
//            t = v_pk_mul_f32(x, v); r = v_pk_add_f32(p, t) (r.lo = p.lo + t.lo), back to back,
//            and counting per lane how often r differs from the same sum done with scalar ops.
// aggressor: 8-wave workgroups, 2 waves per SIMD at <= 208 VGPRs (room for the victim), a loop
//            of v_mfma_f32_16x16x32_f16 chains (the FIR bank's instruction) and a little VALU.
// Modes (argv[1]): 0 = victim alone, 1 = victim beside the aggressor, 2 = victim with its SIMD
// claimed whole (v255 / a255 named) beside the aggressor.  Prints mismatch counts per lane group.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <bool OWN>
__global__ __launch_bounds__(64) void victim(long iters, unsigned* __restrict__ bad,
                                             float* __restrict__ sink) {
    if constexpr (OWN) asm volatile("" ::: "v255", "a255");
    const int lane = threadIdx.x;
    f32x2 x = {1.0f + lane * 1e-3f, 0.5f + lane * 2e-3f};
    f32x2 v = {0.75f - lane * 1e-3f, -0.25f + lane * 1e-3f};
    f32x2 p = {0.125f, -0.5f};
    unsigned nbad = 0;
    float acc = 0.f;
    for (long i = 0; i < iters; ++i) {
        f32x2 t, r;
        asm volatile(
            "v_pk_mul_f32 %[t], %[x], %[v]\n\t"
            "v_pk_add_f32 %[r], %[p], %[t]\n\t"
            : [t] "=&v"(t), [r] "=&v"(r)
            : [x] "v"(x), [v] "v"(v), [p] "v"(p));
        // the same sum with scalar ops (separate instructions, results used much later)
        const float lo = p.x + x.x * v.x, hi = p.y + x.y * v.y;
        nbad += (r.x != lo) | (r.y != hi);
        acc += r.x;
        // vary the operands a little so nothing is loop-invariant
        x.x = x.x * 0.9999999f + 1e-7f;
        v.y = v.y * 0.9999998f + 2e-7f;
    }
    atomicAdd(&bad[blockIdx.x * 64 + lane], nbad);
    sink[blockIdx.x * 64 + lane] = acc;
}

__global__ __launch_bounds__(512) void aggressor(long iters, float* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    f16x8 a, b;
    for (int k = 0; k < 8; ++k) {
        a[k] = (_Float16)(0.01f * (lane + k));
        b[k] = (_Float16)(0.02f * (lane - k));
    }
    f32x4 c[8];
    for (int j = 0; j < 8; ++j) c[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float s = 0.f;
    for (long i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[j], 0, 0, 0);
        s += c[i & 7][0];
        a[0] = (_Float16)((float)a[0] + 1e-3f);
    }
    float t = s;
    for (int j = 0; j < 8; ++j) t += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    sink[blockIdx.x * 512 + threadIdx.x] = t;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 1;
    const int nvb = 16;                 // victim workgroups (one wave each)
    const long viters = argc > 2 ? atol(argv[2]) : 2000000;
    const long aiters = argc > 3 ? atol(argv[3]) : 400000;
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    unsigned* bad;
    float *vs, *as;
    CK(hipMalloc(&bad, nvb * 64 * sizeof(unsigned)));
    CK(hipMemset(bad, 0, nvb * 64 * sizeof(unsigned)));
    CK(hipMalloc(&vs, nvb * 64 * sizeof(float)));
    CK(hipMalloc(&as, (size_t)cus * 512 * sizeof(float)));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s1));
    if (mode == 2) hipLaunchKernelGGL(victim<true>, dim3(nvb), dim3(64), 0, s1, viters, bad, vs);
    else hipLaunchKernelGGL(victim<false>, dim3(nvb), dim3(64), 0, s1, viters, bad, vs);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, s1));
    if (mode >= 1) {
        hipLaunchKernelGGL(aggressor, dim3(cus), dim3(512), 0, s2, aiters, as);
        CK(hipGetLastError());
    }
    CK(hipDeviceSynchronize());
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned> h(nvb * 64);
    CK(hipMemcpy(h.data(), bad, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    unsigned long long grp[4] = {0, 0, 0, 0}, tot = 0;
    for (int b = 0; b < nvb; ++b)
        for (int l = 0; l < 64; ++l) {
            grp[l / 16] += h[b * 64 + l];
            tot += h[b * 64 + l];
        }
    printf("mode %d (%s): victim %.2f ms, %ld pairs per lane; mismatches lanes 0-15 %llu, 16-31 %llu, "
           "32-47 %llu, 48-63 %llu, total %llu\n",
           mode, mode == 0 ? "alone" : (mode == 1 ? "beside MFMA waves" : "own SIMD beside MFMA waves"), ms,
           viters, grp[0], grp[1], grp[2], grp[3], tot);
    return 0;
}
