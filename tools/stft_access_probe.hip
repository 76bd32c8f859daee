// stft_access_probe.hip -- does the 64K STFT's access width matter?  fft64k_pass_a/b
// (fft.hip) move every sample as 8-byte lane accesses in 256-byte row segments 2 KiB apart
// (32 columns of a 256 x 256 frame per workgroup).  This copies 2 GiB (2^28 c64) in -> out
// with the same segment pattern at 8-byte and at 16-byte lane width (two adjacent columns per
// lane, 64 columns per workgroup), and fully linear 16-byte for reference; non-temporal loads
// and stores as in the kernels.  No compute.  HIP events, 20 timed launches after 3 warmups.
// Build: hipcc -O3 --offload-arch=gfx950 stft_access_probe.hip -o stft_access_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr long M = 65536;

// 512 lanes: (j < 16, c < 32), 16 rows each: the pass-A pattern, 8 B per lane
__global__ __launch_bounds__(512) void k_seg8(const f2* __restrict__ in, f2* __restrict__ out) {
    const int c = threadIdx.x % 32, j = threadIdx.x / 32;
    const long f = blockIdx.x / 8;
    const int col = 32 * (blockIdx.x % 8) + c;
    const f2* s = in + f * M;
    f2* d = out + f * M;
    f2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = __builtin_nontemporal_load(s + 256 * (j + 16 * m) + col);
#pragma unroll
    for (int m = 0; m < 16; ++m) __builtin_nontemporal_store(v[m], d + 256 * (j + 16 * m) + col);
}

// 512 lanes: (j < 16, c < 32), two adjacent columns per lane: 16 B, 512-byte row segments
__global__ __launch_bounds__(512) void k_seg16(const f2* __restrict__ in, f2* __restrict__ out) {
    const int c = threadIdx.x % 32, j = threadIdx.x / 32;
    const long f = blockIdx.x / 4;
    const int col = 64 * (blockIdx.x % 4) + 2 * c;
    const f4* s = reinterpret_cast<const f4*>(in + f * M);
    f4* d = reinterpret_cast<f4*>(out + f * M);
    f4 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = __builtin_nontemporal_load(s + (256 * (j + 16 * m) + col) / 2);
#pragma unroll
    for (int m = 0; m < 16; ++m) __builtin_nontemporal_store(v[m], d + (256 * (j + 16 * m) + col) / 2);
}

// linear: 512 lanes x 16 B x 16 per workgroup, contiguous
__global__ __launch_bounds__(512) void k_lin16(const f2* __restrict__ in, f2* __restrict__ out) {
    const f4* s = reinterpret_cast<const f4*>(in) + (long)blockIdx.x * 8192;
    f4* d = reinterpret_cast<f4*>(out) + (long)blockIdx.x * 8192;
    f4 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = __builtin_nontemporal_load(s + 512 * m + threadIdx.x);
#pragma unroll
    for (int m = 0; m < 16; ++m) __builtin_nontemporal_store(v[m], d + 512 * m + threadIdx.x);
}

int main() {
    const long n = 1L << 28;  // c64 samples: 4096 frames of 64K
    f2 *in, *out;
    if (hipMalloc(&in, n * sizeof(f2)) != hipSuccess || hipMalloc(&out, n * sizeof(f2)) != hipSuccess) return 1;
    hipMemset(in, 0, n * sizeof(f2));
    const long frames = n / M;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = 2.0 * n * sizeof(f2);
    for (int var = 0; var < 3; ++var) {
        const char* name = var == 0 ? "seg8 (pass A/B pattern, 8 B lanes, 256 B segments)"
                         : var == 1 ? "seg16 (16 B lanes, 512 B segments)" : "lin16 (contiguous 16 B)";
        float sum = 0.f;
        const int reps = 20;
        for (int rep = 0; rep < reps + 3; ++rep) {
            hipEventRecord(e0);
            if (var == 0) hipLaunchKernelGGL(k_seg8, dim3(frames * 8), dim3(512), 0, 0, in, out);
            else if (var == 1) hipLaunchKernelGGL(k_seg16, dim3(frames * 4), dim3(512), 0, 0, in, out);
            else hipLaunchKernelGGL(k_lin16, dim3(n / 16384), dim3(512), 0, 0, in, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep >= 3) sum += ms;
        }
        const float mean = sum / reps;
        printf("%-55s %.4f ms  %.2f TB/s\n", name, mean, bytes / (mean * 1e-3) / 1e12);
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
