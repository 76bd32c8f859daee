// mfma_window_probe.hip -- round 5 diagnostic (not product): does the matrix instruction's
// operand type change how long a launch takes in the clock dip after an idle gap (the window
// bench.py's 20 timed launches fall in)?  Each arm issues the SAME number of
// 16-cycle MFMAs per wave with operands that change every iteration (fresh bits from a
// per-lane xorshift, so the multiplier inputs toggle like sample data), 8 waves per CU, one
// workgroup per CU, sized to ~0.5 ms at full clock:
//   f16:  v_mfma_f32_16x16x32_f16   (the c64 FIR's instruction)
//   i8:   v_mfma_i32_16x16x64_i8    (the u8 FIR's; twice the K per instruction)
//   f16k16: v_mfma_f32_16x16x16_f16 (half the K of the f16 arm: is it half the cycles?)
// argv[1] = arm, argv[2] = iterations per wave.  Prints per-launch times: 1 s idle, then 25
// launches (the driver's 5 warmup + 20 timed), then 200 back to back.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned xs(unsigned& s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

template <int ARM>
__global__ __launch_bounds__(512) void probe(long iters, float* __restrict__ sink) {
    unsigned s = 0x9e3779b9u * (threadIdx.x + 1) + blockIdx.x * 7919u;
    f32x4 cf[4] = {};
    i32x4 ci[4] = {};
    unsigned a[4], b[4];
    for (int k = 0; k < 4; ++k) {
        a[k] = xs(s) & 0x3bff3bffu;  // fp16 pairs below 1.0 (no inf / nan), a fixed "tap" operand
        b[k] = xs(s);
    }
    for (long i = 0; i < iters; ++i) {
        // fresh B bits every iteration (4 VALU), then 8 MFMAs
        unsigned nb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) nb[k] = xs(s);
        if constexpr (ARM == 0) {
            unsigned m[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = nb[k] & 0x3bff3bffu;
            f16x8 A, B;
            __builtin_memcpy(&A, a, 16);
            __builtin_memcpy(&B, m, 16);
#pragma unroll
            for (int j = 0; j < 8; ++j) cf[j & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, cf[j & 3], 0, 0, 0);
        } else if constexpr (ARM == 2) {
            typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
            unsigned m[2] = {nb[0] & 0x3bff3bffu, nb[1] & 0x3bff3bffu};
            f16x4 A, B;
            __builtin_memcpy(&A, a, 8);
            __builtin_memcpy(&B, m, 8);
#pragma unroll
            for (int j = 0; j < 8; ++j) cf[j & 3] = __builtin_amdgcn_mfma_f32_16x16x16f16(A, B, cf[j & 3], 0, 0, 0);
        } else {
            typedef int i32x4t __attribute__((ext_vector_type(4)));
            i32x4t A, B;
            __builtin_memcpy(&A, a, 16);
            __builtin_memcpy(&B, nb, 16);
#pragma unroll
            for (int j = 0; j < 8; ++j) ci[j & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, ci[j & 3], 0, 0, 0);
        }
    }
    float t = 0.f;
    for (int j = 0; j < 4; ++j) t += cf[j][0] + cf[j][3] + (float)ci[j][0] + (float)ci[j][2];
    sink[blockIdx.x * 512 + threadIdx.x] = t;
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const int arm = argc > 1 ? (strcmp(argv[1], "i8") == 0 ? 1 : strcmp(argv[1], "f16k16") == 0 ? 2 : 0) : 0;
    const long iters = argc > 2 ? atol(argv[2]) : 2000;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float* sink;
    CK(hipMalloc(&sink, (size_t)cus * 512 * sizeof(float)));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int nl = 25 + 200;
    std::vector<hipEvent_t> ev(nl + 1);
    for (auto& e : ev) CK(hipEventCreate(&e));
    auto go = [&]() {
        if (arm == 1) hipLaunchKernelGGL(probe<1>, dim3(cus), dim3(512), 0, st, iters, sink);
        else if (arm == 2) hipLaunchKernelGGL(probe<2>, dim3(cus), dim3(512), 0, st, iters, sink);
        else hipLaunchKernelGGL(probe<0>, dim3(cus), dim3(512), 0, st, iters, sink);
    };
    go();  // load the code object
    CK(hipStreamSynchronize(st));
    std::this_thread::sleep_for(std::chrono::seconds(1));
    CK(hipEventRecord(ev[0], st));
    for (int i = 0; i < nl; ++i) {
        go();
        CK(hipEventRecord(ev[i + 1], st));
    }
    CK(hipStreamSynchronize(st));
    std::vector<float> ms(nl);
    for (int i = 0; i < nl; ++i) CK(hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]));
    double w = 0, l = 0;
    for (int i = 5; i < 25; ++i) w += ms[i];
    for (int i = 25; i < nl; ++i) l += ms[i];
    printf("{\"arm\": \"%s\", \"iters\": %ld, \"driver_window_ms\": %.4f, \"steady_ms\": %.4f, \"first25\": [",
           arm == 1 ? "i8" : arm == 2 ? "f16k16" : "f16", iters, w / 20, l / 200);
    for (int i = 0; i < 25; ++i) printf("%s%.4f", i ? ", " : "", ms[i]);
    printf("]}\n");
    return 0;
}
