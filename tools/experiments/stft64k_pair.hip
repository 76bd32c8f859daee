// stft64k_pair.hip -- experiment (not in libsdrgpu.so): a ONE-PASS 64 Ki-point STFT with
// no scratch slab, sized to what one CU can hold.
//
// Why this shape.  A 64K c64 frame is 512 KiB = the CU's whole VGPR file (4 SIMDs x 512
// regs x 64 lanes x 4 B), so a frame cannot be CU-resident with room left for the FFT's
// working set; every 4-way split that keeps outputs contiguous (DIT) needs all four 16K
// sub-spectra resident at once (512 KiB again).  The split that fits is the radix-4 DIF of
// fft_dif4_kernel with TWO of its four sub-sequences per workgroup:
//   y_m[n] = (sum_p x[n + pM] (-i)^{pm}) W_N^{mn},  X[4k + m] = DFT_M(y_m)[k],  M = N/4,
// workgroup (frame, h) forms y_h and y_{h+2} (h = 0, 1) in one read of the frame: y_h goes to
// LDS (16K points, 136 KiB padded), y_{h+2} stays in VGPRs (32 points per lane at 512 lanes);
// FFT y_h in LDS (Stockham radix 16,16,16,4), store X[4k+h]; move y_{h+2} into LDS, FFT,
// store X[4k+h+2].  Frame reads: 2x (the pair shares them through the XCD's L2; dif4 read
// 4x), stores: 8 B per lane at a 32-B stride (the frame's four sub-FFTs interleave).
//
// Built standalone (own main): hipcc -O3 --offload-arch=gfx950 -o tools/bin/stft64k_pair
// tools/experiments/stft64k_pair.hip.  Run: tools/bin/stft64k_pair [reps]; prints, for the
// full kernel and for a timing-only build without the DFT / twiddle arithmetic (MATH=false:
// same loads, LDS passes, barriers and stores), ms per 2^28-sample STFT and the error of
// three frames against a host double-precision FFT.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../unnamed-rust-sdr_amd/csrc/fft_device.hpp"

using namespace sdrgpu::fftd;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int N = 65536;
constexpr int M = N / 4;
constexpr int NTH = 512;
constexpr int PPT = M / NTH;  // 32 points per lane per pass
__device__ __forceinline__ int fpad(int i) { return i + (i >> 4); }
constexpr int LDS_ELEMS = M + M / 16;

// one Stockham pass of radix R over the M-point sequence in LDS (autosort, natural order out)
template <int R, int NS, bool MATH>
__device__ __forceinline__ void pass(float2* lds, const float2* __restrict__ twN) {
    constexpr int NBF = PPT / R;  // butterflies per lane
    constexpr int BPT = M / R;
    const int t = threadIdx.x;
    float2 v[NBF][R];
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
        const int j = t + NTH * u;
#pragma unroll
        for (int r = 0; r < R; ++r) v[u][r] = lds[fpad(j + r * BPT)];
        if (MATH) {
            if (NS > 1) {
                const int k = j % NS;
                twiddle<R, false>(v[u], twN, 4 * k * (M / (NS * R)));  // W_M^k = W_N^{4k}
            }
            Dft<R, false>::run(v[u]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
        const int j = t + NTH * u;
        const int k = j % NS;
        const int o = (j / NS) * NS * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[fpad(o + r * NS)] = v[u][r];
    }
    __syncthreads();
}

template <bool MATH>
__device__ __forceinline__ void fft16k(float2* lds, const float2* __restrict__ twN) {
    pass<16, 1, MATH>(lds, twN);
    pass<16, 16, MATH>(lds, twN);
    pass<16, 256, MATH>(lds, twN);
    pass<4, 4096, MATH>(lds, twN);
}

// bin 4k + m of frame f, collated (fft.rs: shift by N/2) and scaled
template <int UNUSED = 0>
__device__ __forceinline__ void store_sub(float2* __restrict__ out, long f, int m, const float2* lds,
                                          float norm) {
    float2* O = out + f * (long)N;
#pragma unroll 8
    for (int i = 0; i < PPT; ++i) {
        const int k = threadIdx.x + NTH * i;
        const float2 x = lds[fpad(k)];
        const int o = (4 * k + m + N / 2) & (N - 1);
        O[o] = make_float2(x.x * norm, x.y * norm);
    }
}

// frames f at in + f * hop (hop = N/2): block b -> XCD b % 8; each XCD takes a contiguous
// range of frames, the two workgroups of a frame on consecutive slots of that XCD
template <bool MATH>
__global__ __launch_bounds__(NTH) void stft64k_pair_kernel(const float2* __restrict__ in, long nframes,
                                                           long fpx, const float2* __restrict__ twN,
                                                           float norm, float2* __restrict__ out) {
    extern __shared__ float2 lds[];
    const long b = blockIdx.x;
    const long xcd = b & 7, slot = b >> 3;
    const int h = (int)(slot & 1);
    const long f = xcd * fpx + (slot >> 1);
    if (f >= nframes) return;
    const float2* base = in + f * (long)(N / 2);
    const int t = threadIdx.x;
    float2 keep[PPT];
#pragma unroll 4
    for (int i = 0; i < PPT; ++i) {
        const int n = t + NTH * i;
        float2 x0 = base[n], x1 = base[n + M], x2 = base[n + 2 * M], x3 = base[n + 3 * M];
        if (MATH) {
            dft4<false>(x0, x1, x2, x3);  // x_m = sum_p x[n + pM] (-i)^{pm}
            const float2 ya = h ? cmul(x1, twN[n]) : x0;
            const float2 yb = cmul(h ? x3 : x2, twN[(h ? 3 : 2) * n]);
            lds[fpad(n)] = ya;
            keep[i] = yb;
        } else {
            lds[fpad(n)] = cadd(x0, x1);
            keep[i] = cadd(x2, x3);
        }
    }
    __syncthreads();
    fft16k<MATH>(lds, twN);
    store_sub(out, f, h, lds, norm);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PPT; ++i) lds[fpad(t + NTH * i)] = keep[i];
    __syncthreads();
    fft16k<MATH>(lds, twN);
    store_sub(out, f, h + 2, lds, norm);
}

static void host_fft(std::vector<std::complex<double>>& a) {  // iterative radix-2, forward
    const int n = (int)a.size();
    for (int i = 1, j = 0; i < n; ++i) {
        int bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (int len = 2; len <= n; len <<= 1) {
        const double ang = -2 * M_PI / len;
        for (int i = 0; i < n; i += len)
            for (int k = 0; k < len / 2; ++k) {
                const std::complex<double> w(std::cos(ang * k), std::sin(ang * k));
                const auto u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
    }
}

template <bool MATH>
static float run(const float2* d_in, long nframes, const float2* d_tw, float2* d_out, int reps) {
    const long fpx = (nframes + 7) / 8;
    const dim3 grid((unsigned)(8 * 2 * fpx)), block(NTH);
    const size_t lds = LDS_ELEMS * sizeof(float2);
    CK(hipFuncSetAttribute((const void*)stft64k_pair_kernel<MATH>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const float norm = 1.0f / std::sqrt((float)N);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(stft64k_pair_kernel<MATH>, grid, block, lds, 0, d_in, nframes, fpx, d_tw, norm, d_out);
    CK(hipGetLastError());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(stft64k_pair_kernel<MATH>, grid, block, lds, 0, d_in, nframes, fpx, d_tw, norm, d_out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const long n_in = 1L << 28;
    const long nframes = (n_in - N) / (N / 2) + 1;  // 8191 full frames at hop N/2
    std::vector<float2> h(1 << 20);
    unsigned s = 12345;
    for (auto& v : h) {
        s = s * 1664525u + 1013904223u;
        v.x = ((s >> 8) * (1.0f / 16777216.0f)) - 0.5f;
        s = s * 1664525u + 1013904223u;
        v.y = ((s >> 8) * (1.0f / 16777216.0f)) - 0.5f;
    }
    float2 *d_in, *d_out, *d_tw;
    CK(hipMalloc(&d_in, n_in * sizeof(float2)));
    CK(hipMalloc(&d_out, nframes * (long)N * sizeof(float2)));
    for (long o = 0; o < n_in; o += (long)h.size())
        CK(hipMemcpy(d_in + o, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
    std::vector<float2> tw(N);
    for (int m = 0; m < N; ++m) {
        const double a = -2 * M_PI * m / N;
        tw[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    CK(hipMalloc(&d_tw, N * sizeof(float2)));
    CK(hipMemcpy(d_tw, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice));
    // in 2^28 * 8 B (each sample read by two frames) + out 2 * 2^28 * 8 B: 24 B / input sample
    const double alg = 24.0 * n_in;
    const float ms_math = run<true>(d_in, nframes, d_tw, d_out, reps);
    // check frames 0, nframes/2, nframes-1 against a host double FFT
    double worst = 0;
    for (long f : {0L, nframes / 2, nframes - 1}) {
        std::vector<std::complex<double>> a(N);
        for (int n = 0; n < N; ++n) {
            const float2 v = h[(f * (N / 2) + n) % h.size()];
            a[n] = {v.x, v.y};
        }
        host_fft(a);
        std::vector<float2> g(N);
        CK(hipMemcpy(g.data(), d_out + f * (long)N, N * sizeof(float2), hipMemcpyDeviceToHost));
        double err = 0, rms = 0;
        for (int k = 0; k < N; ++k) {
            const auto ref = a[k] / std::sqrt((double)N);
            const float2 y = g[(k + N / 2) % N];
            err = std::max(err, std::abs(std::complex<double>(y.x, y.y) - ref));
            rms += std::norm(ref);
        }
        worst = std::max(worst, err / std::sqrt(rms / N));
    }
    const float ms_skel = run<false>(d_in, nframes, d_tw, d_out, reps);
    printf("stft64k_pair: %ld frames of 64Ki (hop 32Ki) over 2^28 c64 samples, %d reps\n", nframes, reps);
    printf("  full kernel   %.4f ms  %.2f TB/s algorithmic (frac %.3f of 8 TB/s)  max|err|/rms %.2e\n",
           ms_math, alg / (ms_math * 1e-3) / 1e12, alg / (ms_math * 1e-3) / 8e12, worst);
    printf("  timing-only   %.4f ms  %.2f TB/s algorithmic (no DFT/twiddle arithmetic)\n", ms_skel,
           alg / (ms_skel * 1e-3) / 1e12);
    return worst < 1e-5 ? 0 : 2;
}
