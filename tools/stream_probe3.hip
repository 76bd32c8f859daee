// stream_probe3.hip -- steady-state HBM ceiling for the headline FIR's byte mix (round 3).
// stream_probe2 timed 20 launches after 3 warmups; the product kernel only settles after ~100
// back-to-back launches (bench.py now times 200 after 20), so this probe times every variant
// the same way: 20 warmups, then 200 launches.  Byte mix: 8 B read + 2 B written per sample,
// 2^28 c64 samples, tiles of 1024 samples (8 KiB in -> 2 KiB out), runs of L tiles per wave
// with the 256-sample history re-read at each run start (the fir_mxh stream, no compute).
// Variants: store policy (non-temporal / default / line-complete non-temporal), tiles in
// flight per wave, and calibration streams (read-only, 1:1 copy, write-only).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++20 stream_probe3.hip -o stream_probe3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr long kTileF4 = 512;  // float4 per tile (8 KiB)

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
    const long lane = threadIdx.x & 63, wave = (blockIdx.x * 256L + threadIdx.x) >> 6;
    const long nw = (gridDim.x * 256L) >> 6;
    f32x4 acc = {0, 0, 0, 0};
    for (long b = wave; b * 256 < n4; b += nw)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x4* q = in + b * 256 + k * 64 + lane;
            acc += NT ? __builtin_nontemporal_load(q) : *q;
        }
    if (acc[0] == 1234.5f) out[lane] = acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const f32x4* __restrict__ in, f32x4* __restrict__ out, long n4) {
    const long i0 = blockIdx.x * 256L + threadIdx.x, st = gridDim.x * 256L;
    for (long i = i0; i < n4; i += st) {
        if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
        else out[i] = in[i];
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write(f32x4* __restrict__ out, long n4) {
    const long i0 = blockIdx.x * 256L + threadIdx.x, st = gridDim.x * 256L;
    const f32x4 v = {1, 2, 3, 4};
    for (long i = i0; i < n4; i += st) {
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

// STORE: 0 non-temporal 32-B-per-lane pairs (the product's pattern), 1 default-policy pairs,
// 2 non-temporal line-complete (lane-linear 1 KiB per instruction), 3 default line-complete
template <int DEPTH, int STORE>
__global__ __launch_bounds__(512) void k_runs(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                             long ntiles, int L) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, W = blockDim.x >> 6;
    const long b0 = blockIdx.x * ntiles / gridDim.x, b1 = (blockIdx.x + 1) * ntiles / gridDim.x;
    auto tile_of = [&](long k) { return b0 + ((k / L) * W + wv) * L + (k % L); };
    f32x4 buf[DEPTH][10];
    auto ld = [&](f32x4 (&b)[10], long k) {
        long tt = tile_of(k);
        const bool ok = tt < b1;
        tt = ok ? tt : b0;
#pragma unroll
        for (int q = 0; q < 8; ++q) b[q] = __builtin_nontemporal_load(in + tt * kTileF4 + 64 * q + lane);
        if ((k % L) == 0) {
            const long th = tt > 0 ? tt : 1;
#pragma unroll
            for (int q = 0; q < 2; ++q) b[8 + q] = in[th * kTileF4 - 128 + 64 * q + lane];
        } else {
            b[8] = b[9] = f32x4{0, 0, 0, 0};
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) ld(buf[d], d);
    for (long k = 0;; k += DEPTH) {
        bool done = false;
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long tc = tile_of(k + d);
            if (tc >= b1) { done = true; break; }
            f32x4 a = buf[d][0] + buf[d][1] + buf[d][2] + buf[d][3] + buf[d][8];
            f32x4 b = buf[d][4] + buf[d][5] + buf[d][6] + buf[d][7] + buf[d][9];
            ld(buf[d], k + d + DEPTH);
            const bool line = STORE >= 2;
            f32x4* o = line ? out + tc * 128 + lane : out + tc * 128 + 2 * lane;
            f32x4* o2 = line ? o + 64 : o + 1;
            if (STORE == 0 || STORE == 2) {
                __builtin_nontemporal_store(a, o);
                __builtin_nontemporal_store(b, o2);
            } else {
                *o = a;
                *o2 = b;
            }
        }
        if (done) break;
    }
}

int main(int argc, char** argv) {
    const int warm = 20, iters = argc > 1 ? atoi(argv[1]) : 200;
    const long n = 1L << 28;     // c64 samples
    const long n4 = n * 8 / 16;  // float4 of input
    const long ntiles = n / 1024;
    f32x4 *in, *out;
    hipMalloc(&in, n * 8);
    hipMalloc(&out, n * 8);
    hipMemset(in, 0, n * 8);
    hipMemset(out, 0, n * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < warm; ++i) launch();
        hipEventRecord(a);
        for (int i = 0; i < iters; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= iters;
        printf("%-40s %.4f ms  %6.0f GB/s (%.3f of 8 TB/s)\n", name, ms, bytes / ms / 1e6,
               bytes / ms / 1e6 / 8000.0);
        fflush(stdout);
    };
    timeit("read-only nt (8 B/sample)", 8.0 * n, [&] { hipLaunchKernelGGL(k_read<true>, dim3(4096), dim3(256), 0, 0, in, out, n4); });
    timeit("read-only default", 8.0 * n, [&] { hipLaunchKernelGGL(k_read<false>, dim3(4096), dim3(256), 0, 0, in, out, n4); });
    timeit("copy 1:1 nt (2^27 c64 in, 1 GiB each way)", 8.0 * n, [&] { hipLaunchKernelGGL(k_copy<true>, dim3(4096), dim3(256), 0, 0, in, out, n4 / 2); });
    timeit("copy 1:1 default", 8.0 * n, [&] { hipLaunchKernelGGL(k_copy<false>, dim3(4096), dim3(256), 0, 0, in, out, n4 / 2); });
    timeit("write-only nt (2 B/sample)", 2.0 * n, [&] { hipLaunchKernelGGL(k_write<true>, dim3(4096), dim3(256), 0, 0, out, n4 / 4); });
    timeit("write-only default", 2.0 * n, [&] { hipLaunchKernelGGL(k_write<false>, dim3(4096), dim3(256), 0, 0, out, n4 / 4); });
#define RUNS(D, S, L, NAME)                                                                             \
    timeit("8:2 runs L=" #L " d" #D " " NAME, 10.0 * n,                                                 \
           [&] { hipLaunchKernelGGL((k_runs<D, S>), dim3(cus), dim3(512), 0, 0, in, out, ntiles, L); });
    RUNS(1, 0, 8, "nt pairs (product)")
    RUNS(1, 1, 8, "default pairs")
    RUNS(1, 2, 8, "nt line")
    RUNS(1, 3, 8, "default line")
    RUNS(2, 0, 8, "nt pairs")
    RUNS(2, 1, 8, "default pairs")
    RUNS(1, 0, 16, "nt pairs")
    RUNS(1, 0, 8, "nt pairs (product, again)")
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
