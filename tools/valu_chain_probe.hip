// valu_chain_probe.hip -- cycles per DEPENDENT VALU instruction on gfx950 as a function of
// the number of active lanes (EXEC) and of the number of independent chains interleaved in
// one wave.  Question behind it: the PLL's per-sample chain (pll.hip) is ~170 dependent VALU
// instructions; does a wave with 16 (or fewer) active lanes issue them faster than a full
// wave64, and does a second independent chain in the same wave come for free?
// One workgroup of one wave; s_memtime (core clock) around 4096 chained v_fma_f32.
// Build: hipcc -O3 --offload-arch=gfx950 valu_chain_probe.hip -o valu_chain_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ __launch_bounds__(64) void k_chain(float* out, long long* cyc, int active, int iters) {
    const int lane = threadIdx.x;
    float a[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = 1.0f + lane * 1e-3f + c;
    const float m = 0.999f, k = 1e-4f;
    if (lane < active) {
        long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
#pragma unroll
                for (int c = 0; c < CHAINS; ++c) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[c]) : "v"(m), "v"(k));
            }
        }
        long long t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) cyc[0] = t1 - t0;
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += a[c];
    out[lane] = s;
}

// dependent transcendental (v_exp_f32) and v_sin_f32-like chain: quarter-rate ops
__global__ __launch_bounds__(64) void k_trans(float* out, long long* cyc, int active, int iters) {
    const int lane = threadIdx.x;
    float a = 0.5f + lane * 1e-3f;
    if (lane < active) {
        long long t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) asm volatile("v_exp_f32 %0, %0" : "+v"(a));
        }
        long long t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) cyc[0] = t1 - t0;
    }
    out[lane] = a;
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 64 * sizeof(float));
    hipMalloc(&cyc, sizeof(long long));
    const int iters = 256;  // x16 = 4096 dependent ops per chain
    auto run = [&](const char* name, auto launch, int ops) {
        long long best = 1LL << 60;
        for (int rep = 0; rep < 5; ++rep) {
            launch();
            hipDeviceSynchronize();
            long long c;
            hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
            if (c < best) best = c;
        }
        printf("%-40s %8lld cycles  %.2f cycles per instruction\n", name, best, (double)best / ops);
    };
    for (int act : {64, 48, 32, 16, 8, 1}) {
        char nm[64];
        snprintf(nm, sizeof nm, "fma chain x1, %d lanes", act);
        run(nm, [&] { hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, out, cyc, act, iters); }, 16 * iters);
        snprintf(nm, sizeof nm, "fma chains x2 interleaved, %d lanes", act);
        run(nm, [&] { hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, out, cyc, act, iters); }, 2 * 16 * iters);
        snprintf(nm, sizeof nm, "fma chains x4 interleaved, %d lanes", act);
        run(nm, [&] { hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, out, cyc, act, iters); }, 4 * 16 * iters);
        snprintf(nm, sizeof nm, "exp chain, %d lanes", act);
        run(nm, [&] { hipLaunchKernelGGL(k_trans, dim3(1), dim3(64), 0, 0, out, cyc, act, iters); }, 16 * iters);
    }
    printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
    return 0;
}
