// mfma_shape_probe.hip -- sustained f16 MFMA rate of v_mfma_f32_16x16x32_f16 against
// v_mfma_f32_32x32x16_f16 with the chip full (256 CUs x 8 waves, two per SIMD, as the FIR
// kernels run).  Question behind it: the D = 1 FIR banks are MFMA-count
// bound at a power-limited clock; the 32x32x16 shape does the same MACs in half the
// instructions with half the operand-register reads per MAC -- does it sustain more FLOP/s?
// Same FLOPs per loop iteration in both shapes (8 x 16x16x32 or 4 x 32x32x16), independent
// accumulators, random fp16 operands (a realistic toggle rate).  Timed with HIP events.
// Build: hipcc -O3 --offload-arch=gfx950 mfma_shape_probe.hip -o mfma_shape_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ _Float16 rnd16(unsigned x, bool zero) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return zero ? (_Float16)0.f : (_Float16)((float)(x & 0xffffu) / 32768.f - 1.f);
}

template <int SHAPE>  // 0: 16x16x32 (8 per iteration), 1: 32x32x16 (4 per iteration)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_mfma(float* out, int iters, int zero_ops) {
    const unsigned t = blockIdx.x * 512u + threadIdx.x;
    f16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[0][i] = rnd16(4 * t + i, zero_ops);
        a[1][i] = rnd16(4 * t + i + 77777u, zero_ops);
        b[0][i] = rnd16(4 * t + i + 12345u, zero_ops);
        b[1][i] = rnd16(4 * t + i + 99991u, zero_ops);
    }
    float s = 0.f;
    if constexpr (SHAPE == 0) {
        f32x4 c[8] = {};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
                c[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[r & 1], b[(r >> 1) & 1], c[r], 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) s += c[r][0] + c[r][3];
    } else {
        f32x16 c[4] = {};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                c[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[r & 1], b[(r >> 1) & 1], c[r], 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) s += c[r][0] + c[r][15];
    }
    out[t] = s;
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus;  // one 512-lane workgroup per CU: 8 waves, two per SIMD
    float* out;
    hipMalloc(&out, (size_t)blocks * 512 * sizeof(float));
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double flop = 2.0 * 8 * 8192.0 * iters * 8 * blocks * 64 / 64;  // per launch (both shapes)
    for (int zero = 0; zero < 2; ++zero) {
        for (int shape = 0; shape < 2; ++shape) {
            float best = 1e30f, sum = 0.f;
            const int reps = 10;
            for (int rep = 0; rep < reps + 2; ++rep) {
                hipEventRecord(e0);
                if (shape == 0) hipLaunchKernelGGL(k_mfma<0>, dim3(blocks), dim3(512), 0, 0, out, iters, zero);
                else hipLaunchKernelGGL(k_mfma<1>, dim3(blocks), dim3(512), 0, 0, out, iters, zero);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep >= 2) { sum += ms; if (ms < best) best = ms; }
            }
            const float mean = sum / reps;
            printf("%s operands %s: mean %.3f ms best %.3f ms  %.1f TFLOP/s (mean)\n",
                   zero ? "zero" : "random", shape ? "v_mfma_f32_32x32x16_f16" : "v_mfma_f32_16x16x32_f16",
                   mean, best, flop / (mean * 1e-3) / 1e12);
        }
    }
    hipFree(out);
    return 0;
}
