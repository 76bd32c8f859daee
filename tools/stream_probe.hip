// stream_probe.hip -- HBM ceiling probe for the FIR stream shape (read 8 B, write 2 B per
// sample; 2^28 c64 samples): what read/write mix and access order can reach on this box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));

// grid-stride: each wave reads 4 x 1 KiB consecutive and writes 1 KiB (4:1)
template <int NT>
__global__ __launch_bounds__(256) void k_grid(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
    const long lane = threadIdx.x & 63;
    const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6;
    const long nw = (gridDim.x * 256L) >> 6;
    for (long b = wave; b * 256 < n4; b += nw) {
        f32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x4* q = in + b * 256 + k * 64 + lane;
            acc += (NT & 1) ? __builtin_nontemporal_load(q) : *q;
        }
        f32x4* o = out + b * 64 + lane;
        if (NT & 2) __builtin_nontemporal_store(acc, o); else *o = acc;
    }
}

// wave-contiguous: each wave owns n4/waves consecutive float4, streams 4 KiB per step
template <int NT, int DEPTH>
__global__ __launch_bounds__(256) void k_range(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
    const long lane = threadIdx.x & 63;
    const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6;
    const long nw = (gridDim.x * 256L) >> 6;
    const long per = n4 / nw;  // multiple of 256 assumed
    const long b0 = wave * per / 256, b1 = (wave + 1) * per / 256;
    f32x4 buf[DEPTH][4];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x4* q = in + (b0 + d) * 256 + k * 64 + lane;
            buf[d][k] = (NT & 1) ? __builtin_nontemporal_load(q) : *q;
        }
    for (long b = b0; b < b1; b += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            f32x4 acc = buf[d][0] + buf[d][1] + buf[d][2] + buf[d][3];
            const long bn = (b + d + DEPTH < b1) ? b + d + DEPTH : b0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f32x4* q = in + bn * 256 + k * 64 + lane;
                buf[d][k] = (NT & 1) ? __builtin_nontemporal_load(q) : *q;
            }
            f32x4* o = out + (b + d) * 64 + lane;
            if (NT & 2) __builtin_nontemporal_store(acc, o); else *o = acc;
        }
    }
}

int main() {
    const long n = 1L << 28;        // c64 samples
    const long n4 = n * 8 / 16;     // float4 of input
    f32x4 *in, *out;
    hipMalloc(&in, n * 8);
    hipMalloc(&out, n * 2);
    hipMemset(in, 0, n * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 20;
        printf("%-28s %.4f ms  %.0f GB/s (%.1f%% of 8 TB/s)\n", name, ms, 10.0 * n / ms / 1e6,
               10.0 * n / ms / 1e6 / 80.0);
    };
    for (int blocks : {1024, 2048, 4096, 8192}) {
        char nm[64];
        snprintf(nm, sizeof nm, "grid nt0 blocks=%d", blocks);
        timeit(nm, [&] { hipLaunchKernelGGL(k_grid<0>, dim3(blocks), dim3(256), 0, 0, in, out, n4); });
        snprintf(nm, sizeof nm, "grid nt3 blocks=%d", blocks);
        timeit(nm, [&] { hipLaunchKernelGGL(k_grid<3>, dim3(blocks), dim3(256), 0, 0, in, out, n4); });
    }
    for (int blocks : {256, 512, 1024}) {
        char nm[64];
        snprintf(nm, sizeof nm, "range nt0 d2 blocks=%d", blocks);
        timeit(nm, [&] { hipLaunchKernelGGL((k_range<0, 2>), dim3(blocks), dim3(256), 0, 0, in, out, n4); });
        snprintf(nm, sizeof nm, "range nt3 d2 blocks=%d", blocks);
        timeit(nm, [&] { hipLaunchKernelGGL((k_range<3, 2>), dim3(blocks), dim3(256), 0, 0, in, out, n4); });
        snprintf(nm, sizeof nm, "range nt3 d4 blocks=%d", blocks);
        timeit(nm, [&] { hipLaunchKernelGGL((k_range<3, 4>), dim3(blocks), dim3(256), 0, 0, in, out, n4); });
    }
    return 0;
}
