// stream_probe4.hip -- cache-policy sweep of the headline FIR's byte mix (round 3).
// Same stream as stream_probe3's "8:2 runs L=8 d1 nt line" (2^28 c64 samples, 8 KiB tiles,
// runs of 8 tiles per wave, 8 waves per CU, 256-sample history re-read per run, line-complete
// 16-B stores), but every load and store goes through the buffer intrinsics so the cache-
// policy bits can be chosen: aux bit 0 = sc0, bit 1 = nt, bit 4 = sc1 (gfx940-family CPol).
// 20 warmups, then ITERS (default 200) timed launches per variant.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++20 stream_probe4.hip -o stream_probe4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr long kTileB = 8192;  // bytes per tile

template <int LP, int SP, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_mix(const char* __restrict__ in, char* __restrict__ out,
                                                  long ntiles, int L) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, W = WPB;
    const long b0 = blockIdx.x * ntiles / gridDim.x, b1 = (blockIdx.x + 1) * ntiles / gridDim.x;
#define tile_of(k) (b0 + (((k) / L) * W + wv) * L + ((k) % L))
    // one descriptor per workgroup range (< 2^31 bytes either way)
    const __amdgpu_buffer_rsrc_t rin =
        __builtin_amdgcn_make_buffer_rsrc((void*)(in + b0 * kTileB - 2048), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout =
        __builtin_amdgcn_make_buffer_rsrc((void*)(out + b0 * (kTileB / 4)), 0, 0x7fffffff, 0x00020000);
    u32x4 buf[10];
    // (no lambdas: a descriptor captured by reference lands in scratch)
#define LD(K)                                                                                      \
    {                                                                                              \
        long tt = tile_of(K);                                                                      \
        tt = tt < b1 ? tt : b0;                                                                    \
        const int base = (int)((tt - b0) * kTileB) + 2048;                                         \
        _Pragma("unroll") for (int q = 0; q < 8; ++q)                                              \
            buf[q] = __builtin_amdgcn_raw_buffer_load_b128(rin, base + 1024 * q + 16 * lane, 0, LP); \
        if (((K) % L) == 0) {                                                                      \
            _Pragma("unroll") for (int q = 0; q < 2; ++q)                                          \
                buf[8 + q] = __builtin_amdgcn_raw_buffer_load_b128(rin, base - 2048 + 1024 * q + 16 * lane, 0, 0); \
        } else {                                                                                   \
            buf[8] = buf[9] = u32x4{0, 0, 0, 0};                                                   \
        }                                                                                          \
    }
    LD(0)
    for (long k = 0;; ++k) {
        const long tc = tile_of(k);
        if (tc >= b1) break;
        u32x4 a = buf[0] + buf[1] + buf[2] + buf[3] + buf[8];
        u32x4 b = buf[4] + buf[5] + buf[6] + buf[7] + buf[9];
        LD(k + 1)
        const int ob = (int)((tc - b0) * (kTileB / 4)) + 16 * lane;
        __builtin_amdgcn_raw_buffer_store_b128(a, rout, ob, 0, SP);
        __builtin_amdgcn_raw_buffer_store_b128(b, rout, ob + 1024, 0, SP);
    }
#undef LD
}

int main(int argc, char** argv) {
    const int warm = 20, iters = argc > 1 ? atoi(argv[1]) : 200;
    const long n = 1L << 28;  // c64 samples
    const long ntiles = n / 1024;
    char *in, *out;
    hipMalloc(&in, n * 8 + 4096);
    hipMalloc(&out, n * 8);
    hipMemset(in, 0, n * 8 + 4096);
    hipMemset(out, 0, n * 8);
    in += 2048;  // the first run's history re-read stays inside the allocation
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
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= iters;
        printf("%-44s %.4f ms  %6.0f GB/s (%.3f of 8 TB/s)\n", name, ms, bytes / ms / 1e6,
               bytes / ms / 1e6 / 8000.0);
        fflush(stdout);
    };
#define MIX(LP, SP, W, G, NAME)                                                                        \
    timeit("load " #LP " store " #SP " " #W "w grid " #G " " NAME, 10.0 * n, [&] {                    \
        hipLaunchKernelGGL((k_mix<LP, SP, W>), dim3(G), dim3(64 * W), 0, 0, in, out, ntiles, 8);      \
    });
    MIX(2, 2, 8, cus, "(nt / nt: the product's policy)")
    MIX(2, 0, 8, cus, "")
    MIX(2, 16, 8, cus, "(store sc1)")
    MIX(2, 17, 8, cus, "(store sc0 sc1)")
    MIX(2, 18, 8, cus, "(store sc1 nt)")
    MIX(2, 3, 8, cus, "(store sc0 nt)")
    MIX(2, 19, 8, cus, "(store sc0 sc1 nt)")
    MIX(0, 2, 8, cus, "(load default)")
    MIX(3, 2, 8, cus, "(load sc0 nt)")
    MIX(18, 2, 8, cus, "(load sc1 nt)")
    MIX(19, 2, 8, cus, "(load sc0 sc1 nt)")
    MIX(2, 2, 12, cus, "")
    MIX(2, 2, 16, cus, "")
    MIX(2, 2, 8, 2 * cus, "")
    MIX(2, 2, 4, 2 * cus, "")
    MIX(2, 2, 8, cus, "(nt / nt again)")
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
