// stream_probe2.hip -- HBM ceiling for the headline FIR's byte mix (read 8 B, write 2 B per
// sample, 2^28 c64 samples), round 2: register streaming vs LDS-DMA (global_load_lds_dwordx4)
// streaming with a per-wave ring, at several waves per CU and ring depths.  Each "tile" is
// 8 KiB of input (1024 samples) -> 2 KiB of output, the fir_mxh tile shape.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++20 stream_probe2.hip -o stream_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr long kTileF4 = 512;  // float4 per tile (8 KiB)

// read-only / write-only calibration (grid-stride, 1 KiB per wave-instruction)
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

__global__ __launch_bounds__(256) void k_write(f32x4* __restrict__ out, long n4) {
    const long i0 = blockIdx.x * 256L + threadIdx.x, st = gridDim.x * 256L;
    const f32x4 v = {1, 2, 3, 4};
    for (long i = i0; i < n4; i += st) __builtin_nontemporal_store(v, out + i);
}

__global__ __launch_bounds__(256) void k_write_def(f32x4* __restrict__ out, long n4) {
    const long i0 = blockIdx.x * 256L + threadIdx.x, st = gridDim.x * 256L;
    const f32x4 v = {1, 2, 3, 4};
    for (long i = i0; i < n4; i += st) out[i] = v;
}

// register streaming, per-wave contiguous tile ranges, DEPTH tiles in flight per wave
template <int DEPTH>
__global__ __launch_bounds__(512) void k_vgpr(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                             long ntiles) {
    const int lane = threadIdx.x & 63;
    const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
    const long nw = (gridDim.x * (long)blockDim.x) >> 6;
    const long t0 = wave * ntiles / nw, t1 = (wave + 1) * ntiles / nw;
    f32x4 buf[DEPTH][8];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int k = 0; k < 8; ++k)
            buf[d][k] = __builtin_nontemporal_load(in + (t0 + d < t1 ? t0 + d : t0) * kTileF4 + 64 * k + lane);
    for (long t = t0; t < t1; t += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            if (t + d >= t1) break;
            f32x4 a = buf[d][0] + buf[d][1] + buf[d][2] + buf[d][3];
            f32x4 b = buf[d][4] + buf[d][5] + buf[d][6] + buf[d][7];
            const long tn = t + d + DEPTH < t1 ? t + d + DEPTH : t0;
#pragma unroll
            for (int k = 0; k < 8; ++k) buf[d][k] = __builtin_nontemporal_load(in + tn * kTileF4 + 64 * k + lane);
            f32x4* o = out + (t + d) * 128 + 2 * lane;
            __builtin_nontemporal_store(a, o);
            __builtin_nontemporal_store(b, o + 1);
        }
    }
}

// register streaming, COOP: the workgroup shares one contiguous range (wave w takes tiles
// w, w+W, ...); HIST: each tile also re-reads the 256 samples before it (the FIR history a
// wave would need when its tiles are not adjacent; L2 hits when the neighbour loaded them)
template <int DEPTH, bool HIST>
__global__ __launch_bounds__(512) void k_vgpr_coop(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                                  long ntiles) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, W = blockDim.x >> 6;
    const long b0 = blockIdx.x * ntiles / gridDim.x, b1 = (blockIdx.x + 1) * ntiles / gridDim.x;
    const long t0 = b0 + wv;
    constexpr int NL = HIST ? 10 : 8;
    f32x4 buf[DEPTH][NL];
    auto ld = [&](f32x4 (&b)[NL], long t) {
        const long tt = t < b1 ? t : t0;
#pragma unroll
        for (int k = 0; k < 8; ++k) b[k] = __builtin_nontemporal_load(in + tt * kTileF4 + 64 * k + lane);
        if (HIST) {
            const long th = tt > 0 ? tt : 1;
#pragma unroll
            for (int k = 0; k < 2; ++k) b[8 + k] = in[th * kTileF4 - 128 + 64 * k + lane];
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) ld(buf[d], t0 + d * W);
    for (long t = t0; t < b1; t += DEPTH * W) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long tc = t + d * W;
            if (tc >= b1) break;
            f32x4 a = buf[d][0] + buf[d][1] + buf[d][2] + buf[d][3];
            f32x4 b = buf[d][4] + buf[d][5] + buf[d][6] + buf[d][7];
            if (HIST) a += buf[d][8] + buf[d][9];
            ld(buf[d], tc + DEPTH * W);
            f32x4* o = out + tc * 128 + 2 * lane;
            __builtin_nontemporal_store(a, o);
            __builtin_nontemporal_store(b, o + 1);
        }
    }
}

// register streaming in RUNS: the workgroup's range is cut into runs of L tiles; wave w takes
// runs w, w+W, ... (so the CU's waves work on W adjacent runs at a time) and re-reads the
// 256 samples before each run (history); prefetch crosses run boundaries
template <int DEPTH>
__global__ __launch_bounds__(512) void k_vgpr_runs(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                                  long ntiles, int L) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, W = blockDim.x >> 6;
    const long b0 = blockIdx.x * ntiles / gridDim.x, b1 = (blockIdx.x + 1) * ntiles / gridDim.x;
    // k-th tile of this wave: run (k / L) * W + wv, tile k % L inside it
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
            f32x4* o = out + tc * 128 + 2 * lane;
            __builtin_nontemporal_store(a, o);
            __builtin_nontemporal_store(b, o + 1);
        }
        if (done) break;
    }
}

// LDS-DMA streaming: per-wave ring of RING tiles (8 KiB each) in LDS; tile t+RING is issued
// right after tile t is consumed; counted vmcnt (stores count too: 2 stores + 8 DMAs per tile)
// COOP: the workgroup's waves share one contiguous range (wave w takes tiles w, w+W, ...):
// one HBM stream per CU instead of one per wave.  LINE: each store instruction writes 1 KiB
// contiguous (lane-linear) instead of the FIR's 32-B-per-lane pairs.
template <int RING, int WPB, bool COOP = false, bool LINE = false>
__global__ __launch_bounds__(64 * WPB) void k_glds(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                                  long ntiles) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    long t0, t1, ts;
    if (COOP) {
        const long b0 = blockIdx.x * ntiles / gridDim.x, b1 = (blockIdx.x + 1) * ntiles / gridDim.x;
        t0 = b0 + wv;
        t1 = b1;
        ts = WPB;
    } else {
        const long wave = (long)blockIdx.x * WPB + wv;
        const long nw = (long)gridDim.x * WPB;
        t0 = wave * ntiles / nw;
        t1 = (wave + 1) * ntiles / nw;
        ts = 1;
    }
    char* ring = smem + wv * RING * 8192;
    auto issue = [&](long t, int slot) {
        const long tt = t < t1 ? t : t0;  // past the end: a harmless re-read (keeps counts fixed)
        const f32x4* src = in + tt * kTileF4 + lane;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            __builtin_amdgcn_global_load_lds((const void*)(src + 64 * k),
                                             (__attribute__((address_space(3))) void*)(ring + slot * 8192 + 1024 * k),
                                             16, 0, 2);
    };
#pragma unroll
    for (int d = 0; d < RING; ++d) issue(t0 + d * ts, d);
    int slot = 0;
    for (long t = t0; t < t1; t += ts) {
        // everything issued after tile t's DMAs: (RING - 1) iterations x (2 stores + 8 DMAs)
        if constexpr (RING == 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else if constexpr (RING == 3) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
        const f32x4* r = reinterpret_cast<const f32x4*>(ring + slot * 8192) + lane;
        f32x4 a = r[0] + r[64] + r[128] + r[192];
        f32x4 b = r[256] + r[320] + r[384] + r[448];
        f32x4* o = LINE ? out + t * 128 + lane : out + t * 128 + 2 * lane;
        __builtin_nontemporal_store(a, o);
        __builtin_nontemporal_store(b, o + (LINE ? 64 : 1));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the slot refills
        issue(t + RING * ts, slot);
        slot = slot + 1 == RING ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
    const long n = 1L << 28;        // c64 samples
    const long n4 = n * 8 / 16;     // float4 of input
    const long ntiles = n / 1024;
    f32x4 *in, *out;
    hipMalloc(&in, n * 8);
    hipMalloc(&out, n * 8);
    hipMemset(in, 0, n * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(a);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 20;
        printf("%-34s %.4f ms  %6.0f GB/s (%.1f%% of 8 TB/s)\n", name, ms, bytes / ms / 1e6,
               bytes / ms / 1e6 / 80.0);
        fflush(stdout);
    };
    for (int blocks : {1024, 4096})  {
        char nm[64];
        snprintf(nm, sizeof nm, "read-only nt blocks=%d", blocks);
        timeit(nm, 8.0 * n, [&] { hipLaunchKernelGGL(k_read<true>, dim3(blocks), dim3(256), 0, 0, in, out, n4); });
        snprintf(nm, sizeof nm, "read-only blocks=%d", blocks);
        timeit(nm, 8.0 * n, [&] { hipLaunchKernelGGL(k_read<false>, dim3(blocks), dim3(256), 0, 0, in, out, n4); });
    }
    timeit("write-only nt", 2.0 * n, [&] { hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, 0, out, n4 / 4); });
    for (int wpc : {4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "vgpr d1 %d waves/CU", wpc);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL(k_vgpr<1>, dim3(cus), dim3(64 * wpc), 0, 0, in, out, ntiles); });
        snprintf(nm, sizeof nm, "vgpr d2 %d waves/CU", wpc);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL(k_vgpr<2>, dim3(cus), dim3(64 * wpc), 0, 0, in, out, ntiles); });
    }
    for (int wpc : {4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "vgpr coop d1 %d waves/CU", wpc);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_vgpr_coop<1, false>), dim3(cus), dim3(64 * wpc), 0, 0, in, out, ntiles); });
        snprintf(nm, sizeof nm, "vgpr coop d2 %d waves/CU", wpc);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_vgpr_coop<2, false>), dim3(cus), dim3(64 * wpc), 0, 0, in, out, ntiles); });
        snprintf(nm, sizeof nm, "vgpr coop+hist d1 %d waves/CU", wpc);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_vgpr_coop<1, true>), dim3(cus), dim3(64 * wpc), 0, 0, in, out, ntiles); });
    }
    for (int L : {1, 2, 4, 8, 16, 32}) {
        char nm[64];
        snprintf(nm, sizeof nm, "vgpr runs L=%d d1 8w", L);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_vgpr_runs<1>), dim3(cus), dim3(512), 0, 0, in, out, ntiles, L); });
    }
    for (int L : {4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "vgpr runs L=%d d2 8w", L);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_vgpr_runs<2>), dim3(cus), dim3(512), 0, 0, in, out, ntiles, L); });
        snprintf(nm, sizeof nm, "vgpr runs L=%d d2 4w", L);
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_vgpr_runs<2>), dim3(cus), dim3(256), 0, 0, in, out, ntiles, L); });
    }
    timeit("vgpr d2 2x8 waves/CU", 10.0 * n, [&] { hipLaunchKernelGGL(k_vgpr<2>, dim3(2 * cus), dim3(512), 0, 0, in, out, ntiles); });
    timeit("write-only default", 2.0 * n, [&] { hipLaunchKernelGGL(k_write_def, dim3(4096), dim3(256), 0, 0, out, n4 / 4); });
#define GL(R, W, C, L, G)                                                                          \
    {                                                                                               \
        char nm[64];                                                                                \
        snprintf(nm, sizeof nm, "glds ring%d %dw %s%s grid%d", R, W, C ? "coop " : "", L ? "line" : "", G); \
        const size_t lds = (size_t)R * W * 8192;                                                    \
        hipFuncSetAttribute((const void*)k_glds<R, W, C, L>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        timeit(nm, 10.0 * n, [&] { hipLaunchKernelGGL((k_glds<R, W, C, L>), dim3(G), dim3(64 * W), lds, 0, in, out, ntiles); }); \
    }
    GL(4, 2, false, false, cus) GL(4, 2, false, true, cus) GL(8, 1, false, false, cus) GL(6, 2, false, false, cus)
    GL(8, 2, false, false, cus) GL(4, 4, true, false, cus) GL(4, 4, true, true, cus) GL(3, 6, true, false, cus)
    GL(4, 2, true, false, cus) GL(2, 8, true, false, cus) GL(4, 4, false, false, cus / 2) GL(4, 2, false, false, 2 * cus)
    GL(8, 2, true, false, cus) GL(4, 4, false, true, cus)
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
