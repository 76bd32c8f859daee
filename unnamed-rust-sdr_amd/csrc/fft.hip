// fft.hip -- batched Stockham FFT, four-step large FFT and STFT framing for gfx950.
//
// Semantics: fft::fft (reference src/fft.rs:3-28): forward DFT X[k] = sum x[n] e^{-2 pi i kn/N}
// (rustfft FFTplanner::new(false)), then collated out[i] = X[(i - N/2) mod N] * (1/sqrt(N))
// with the norm computed in f32 (fft.rs:16); rfft (fft.rs:30-37) keeps out[N/2..].  The STFT
// framing is Window(N) + Decimate(hop) (src/signal/adapters/mod.rs:270-303, 13-41): frame j
// covers stream samples [(j+1)hop - N, (j+1)hop), zero before the stream start.
//
// Kernels (256 lanes, 16 complex points per lane = one 4096-point LDS tile per workgroup):
//   fft_tile_kernel  -- 4096/M transforms of size M <= 4096 per workgroup: coalesced load
//                       (frame gather folded in), up to 3 radix-{2,4,8,16} Stockham passes in
//                       LDS (twiddles from a 4096-entry table + recurrence), collated store.
//   four-step (M > 4096, M = M1*M2): pass A = M2-point column FFTs on 4096/M2 columns per
//                       workgroup (rows of 4096/M2 contiguous samples -> coalesced), times
//                       W_M^{n1 k2}, to a scratch slab; pass B = M1-point FFTs over n1 on
//                       4096/M1 consecutive k2, collated (shift + 1/sqrt(M)) store.  Frames are
//                       processed in batches whose scratch slab stays in the 256 MiB MALL.
// Roofline: HBM bound (C3: 24 algorithmic bytes per input sample, ~160 flop), see DESIGN.md.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "fft_device.hpp"
#include "fft_frames.hpp"
#include "fft_kernels.hpp"

namespace sdrgpu {

using namespace fftd;

namespace {

constexpr int kFftBlock = 256;
constexpr int kTile = 4096;
__device__ __forceinline__ int fpad(int i) { return i + (i >> 4); }
constexpr int kTileLds = kTile + kTile / 16;

}  // namespace

namespace {

// -------- in-place Stockham pass over the 4096-point tile (all sizes compile-time) -----
// batch of 4096/M transforms of size M; radix R; stride NS.  Each lane does 16/R butterflies.
template <int R, int M, int NS, bool INV>
__device__ __forceinline__ void tile_pass(float2* lds, const float2* __restrict__ tw) {
    constexpr int NBF = 16 / R;
    constexpr int BPT = M / R;  // butterflies per transform
    const int t = threadIdx.x;
    float2 v[NBF][R];
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
        const int g = t * NBF + u;
        const int f = g / BPT, j = g % BPT;   // compile-time power-of-two divisors -> shifts
        const int base = f * M;
#pragma unroll
        for (int r = 0; r < R; ++r) v[u][r] = lds[fpad(base + j + r * BPT)];
        if (NS > 1) {
            const int k = j % NS;
            twiddle<R, INV>(v[u], tw, k * (kTile / (NS * R)));
        }
        Dft<R, INV>::run(v[u]);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
        const int g = t * NBF + u;
        const int f = g / BPT, j = g % BPT;
        const int k = j % NS;
        const int o = f * M + (j / NS) * NS * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[fpad(o + r * NS)] = v[u][r];
    }
    __syncthreads();
}

// radix plan: 16s first, then the remainder (M = 16^a * rem, rem in {1,2,4,8})
template <int M, int NS, bool INV>
__device__ __forceinline__ void tile_fft_rec(float2* lds, const float2* __restrict__ tw) {
    if constexpr (NS < M) {
        constexpr int LEFT = M / NS;
        constexpr int R = LEFT >= 16 ? 16 : LEFT;
        tile_pass<R, M, NS, INV>(lds, tw);
        tile_fft_rec<M, NS * R, INV>(lds, tw);
    }
}

template <int M, bool INV>
__device__ __forceinline__ void tile_fft(float2* lds, const float2* __restrict__ tw) {
    tile_fft_rec<M, 1, INV>(lds, tw);
}

struct TileArgs {
    FrameSrc src;
    long nframes;      // frames this launch
    int M;
    const float2* tw;  // W_4096
    float norm;        // 1/sqrt(M) (f32, fft.rs:16)
    int store_mode;    // 0: collated (fft), 1: upper half of collated (rfft)
    float2* out;
};

template <int M>
__global__ __launch_bounds__(kFftBlock) void fft_tile_kernel(TileArgs a) {
    __shared__ float2 lds[kTileLds];
    const int t = threadIdx.x;
    const int fpt = kTile / M;  // frames per tile
    const long f0 = (long)blockIdx.x * fpt;
    const int nf = (int)min((long)fpt, a.nframes - f0);
    // coalesced load: point p -> (frame p / M, sample p % M), all 16 loads in flight
    {
        float2 v[16];
        gather_tile_ct<16, kFftBlock, M, kTile>(a.src, f0, nf, v);
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[fpad(t + kFftBlock * i)] = v[i];
    }
    __syncthreads();
    tile_fft<M, false>(lds, a.tw);
    if ((a.store_mode == 0 || a.store_mode == 3) && nf == fpt) {
        // full tile: output (f, o) is element p = f M + o of the tile's contiguous output run,
        // a 32-bit offset off one scalar base; every LDS read issued before the first store
        const bool db = a.store_mode == 3;
        char* base = reinterpret_cast<char*>(a.out) + f0 * M * (db ? 4 : 8);
        float2 x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int p = t + kFftBlock * i, o = p % M;
            x[i] = lds[fpad(o + M / 2 < M ? p + M / 2 : p + M / 2 - M)];
        }
        if (db) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                *reinterpret_cast<float*>(base + (unsigned)(t + kFftBlock * i) * 4u) = db_of(x[i], a.norm);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                *reinterpret_cast<float2*>(base + (unsigned)(t + kFftBlock * i) * 8u) =
                    make_float2(x[i].x * a.norm, x[i].y * a.norm);
        }
    } else if (a.store_mode == 0 || a.store_mode == 3) {
        // collated store, output-ordered (coalesced): out[f][i] = X[(i + M/2) % M] * norm
        const int half = M / 2;
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const int p = t + kFftBlock * i;
            const int f = p / M, o = p % M;
            if (f < nf) {
                int k = o + half;
                if (k >= M) k -= M;
                float2 x = lds[fpad(f * M + k)];
                if (a.store_mode == 0) a.out[(f0 + f) * M + o] = make_float2(x.x * a.norm, x.y * a.norm);
                else reinterpret_cast<float*>(a.out)[(f0 + f) * M + o] = db_of(x, a.norm);
            }
        }
    } else {
#pragma unroll 4
        for (int i = 0; i < 16; ++i) {
            const int p = t + kFftBlock * i;
            const int f = p / M, k = p % M;
            if (f < nf) store_bin(a.out, f0 + f, M, k, lds[fpad(f * M + k)], a.store_mode, a.norm);
        }
    }
}

// -------- four-step, pass A: M2-point FFTs down the columns n1 of x[n1 + M1 n2] ---------
struct FourArgs {
    FrameSrc src;
    long nframes;
    int M, M1, M2;
    const float2* tw;       // W_4096
    const float2* twM;      // W_M, M entries
    float norm;
    int store_mode;
    float2* scratch;        // nframes x M: S[f][n1 * M2 + k2]
    float2* out;
};

template <int M2>
__global__ __launch_bounds__(kFftBlock) void fft4_pass_a(FourArgs a) {
    __shared__ float2 lds[kTileLds];
    const int t = threadIdx.x;
    constexpr int C = kTile / M2;                // columns per workgroup
    const int tiles_per_frame = a.M1 / C;
    const long f = blockIdx.x / tiles_per_frame;
    const int c0 = (int)(blockIdx.x % tiles_per_frame) * C;
    if (f >= a.nframes) return;
    // load: point p -> (n2 = p / C, col = p % C): row n2 holds C contiguous samples
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int p = t + kFftBlock * i;
        const int n2 = p / C, col = p % C;
        const float2 x = frame_sample(a.src, a.M, f, (long)(c0 + col) + (long)a.M1 * n2);
        lds[fpad(col * M2 + n2)] = x;             // column-major: transform per column
    }
    __syncthreads();
    tile_fft<M2, false>(lds, a.tw);
    // twiddle W_M^{n1 k2}, store S[n1][k2] (consecutive k2 contiguous)
    float2* S = a.scratch + f * (long)a.M;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int p = t + kFftBlock * i;
        const int col = p / M2, k2 = p % M2;
        const int n1 = c0 + col;
        float2 x = lds[fpad(col * M2 + k2)];
        const int e = (n1 * k2) & (a.M - 1);      // M is a power of two
        x = cmul(x, a.twM[e]);
        S[(long)n1 * M2 + k2] = x;
    }
}

// -------- four-step, pass B: M1-point FFTs over n1 for 4096/M1 consecutive k2 ----------
template <int M1>
__global__ __launch_bounds__(kFftBlock) void fft4_pass_b(FourArgs a) {
    __shared__ float2 lds[kTileLds];
    const int t = threadIdx.x;
    constexpr int C = kTile / M1;                // k2 columns per workgroup
    const int tiles_per_frame = a.M2 / C;
    const long f = blockIdx.x / tiles_per_frame;
    const int c0 = (int)(blockIdx.x % tiles_per_frame) * C;
    if (f >= a.nframes) return;
    const float2* S = a.scratch + f * (long)a.M;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int p = t + kFftBlock * i;
        const int n1 = p / C, col = p % C;
        lds[fpad(col * M1 + n1)] = S[(long)n1 * a.M2 + c0 + col];
    }
    __syncthreads();
    tile_fft<M1, false>(lds, a.tw);
    // X[k2 + M2 k1] by store mode; lanes walk k2 (contiguous)
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int p = t + kFftBlock * i;
        const int k1 = p / C, col = p % C;
        const long k = (long)(c0 + col) + (long)a.M2 * k1;
        store_bin(a.out, f, a.M, k, lds[fpad(col * M1 + k1)], a.store_mode, a.norm);
    }
}


// -------- 65536-point four-step (256 x 256) with wide LDS tiles ---------------------------
// n = 256 r + col, k = k1 + 256 k2.  Pass A: for CB columns per workgroup, FFT-256 over r
// (r = j + 16 m: DFT16 over m in registers, x W_256^{j ka}, LDS transpose, DFT16 over j),
// x W_65536^{col k1}, store S[k1][col] (lanes walk col).  Pass B: for CB consecutive k1
// per workgroup, rows S[k1][*] are read contiguously into LDS, FFT-256 over col the same
// way, and the collated output rows are written with lanes walking k1 (8*CB bytes per k2).
// Global accesses are 8*CB-byte runs (the generic path above moves 128-byte runs); LDS
// accesses are conflict-free (8-byte lanes, padded row pitch in B).
// CB = columns (pass A) / k1 rows (pass B) per workgroup: 16*CB lanes, each lane one
// (j, column) pair; CB = 32 -> 64 KiB (A) / 66 KiB (B) of LDS, two workgroups per CU.
struct F64Args {
    FrameSrc src;
    long nframes;
    const float2* tw;   // W_4096
    const float2* twM;  // W_65536
    float norm;
    int store_mode;
    float2* scratch;
    float2* out;
};

template <typename T> __device__ __forceinline__ T ld_nt(const T* p) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 r = __builtin_nontemporal_load(reinterpret_cast<const f2*>(p));
    return make_float2(r[0], r[1]);
}
__device__ __forceinline__ void st_nt(float2* p, float2 v) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 r = {v.x, v.y};
    __builtin_nontemporal_store(r, reinterpret_cast<f2*>(p));
}

// NT: non-temporal hint on the streamed frame loads (pass A) and output stores (pass B), so
// the stream does not evict the MALL-resident scratch slab
template <int CB, bool NT>
__global__ __launch_bounds__(16 * CB) void fft64k_pass_a(F64Args a) {
    __shared__ float2 lds[16 * 16 * CB];
    constexpr long M = 65536;
    constexpr int NB = 256 / CB;  // workgroups per frame
    const int c = threadIdx.x % CB, j = threadIdx.x / CB;
    const long f = blockIdx.x / NB;
    const int col = CB * (int)(blockIdx.x % NB) + c;
    if (f >= a.nframes) return;
    float2 v[16];
    // frame f samples n = 256 (j + 16 m) + col
    const FrameSrc& s = a.src;
    long g0 = 0;
    bool fast = s.mode == 0;
    if (s.mode == 1) {  // (u8 streams, mode 3, take the generic frame_sample path)
        g0 = s.first_end + f * s.hop - M;
        fast = g0 >= 0 && g0 + M <= s.n_in;
    }
    if (fast) {
        const float2* src = s.mode == 0 ? s.in + f * M : s.in + g0;
#pragma unroll
        for (int m = 0; m < 16; ++m)
            v[m] = NT ? ld_nt(src + 256 * (j + 16 * m) + col) : src[256 * (j + 16 * m) + col];
    } else {
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = frame_sample(s, M, f, 256 * (j + 16 * m) + col);
    }
    Dft<16, false>::run(v);
    if (j) twiddle<16, false>(v, a.tw, 16 * j);
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) lds[(ka * 16 + j) * CB + c] = v[ka];
    __syncthreads();
    const int ka = j;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = lds[(ka * 16 + jj) * CB + c];
    Dft<16, false>::run(v);
    // v[kb] = column FFT at k1 = ka + 16 kb; x W_65536^{col k1} = W^{col ka} (W_4096^{col})^kb
    const float2 w1 = a.twM[col * ka];
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) v[kb] = cmul(v[kb], w1);
    twiddle<16, false>(v, a.tw, col);
    float2* S = a.scratch + f * M;
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) S[(long)(ka + 16 * kb) * 256 + col] = v[kb];
}

template <int CB, bool NT>
__global__ __launch_bounds__(16 * CB) void fft64k_pass_b(F64Args a) {
    constexpr int P = CB + 1;  // LDS row pitch (float2): conflict-free transposes
    __shared__ float2 lds[256 * P];
    constexpr long M = 65536;
    constexpr int NB = 256 / CB;
    constexpr int NTH = 16 * CB;
    const int t = threadIdx.x;
    const long f = blockIdx.x / NB;
    const int k1b = CB * (int)(blockIdx.x % NB);
    if (f >= a.nframes) return;
    const float2* S = a.scratch + f * M + (long)k1b * 256;
    // rows k1b + r (r < CB), 256 columns each: coalesced, transposed into lds[col][r]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int p = t + NTH * i;
        const int r = p >> 8, col = p & 255;
        lds[col * P + r] = S[p];
    }
    __syncthreads();
    const int r = t % CB, j = t / CB;
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = lds[(j + 16 * m) * P + r];
    __syncthreads();
    Dft<16, false>::run(v);
    if (j) twiddle<16, false>(v, a.tw, 16 * j);
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) lds[(ka * 16 + j) * P + r] = v[ka];
    __syncthreads();
    const int ka = j;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = lds[(ka * 16 + jj) * P + r];
    Dft<16, false>::run(v);
    // X[k1 + 256 k2] with k1 = k1b + r, k2 = ka + 16 kb -> collated out[(k + M/2) mod M]
    if (a.store_mode != 0) {
#pragma unroll
        for (int kb = 0; kb < 16; ++kb)
            store_bin(a.out, f, M, (long)(k1b + r) + 256L * (ka + 16 * kb), v[kb], a.store_mode, a.norm);
        return;
    }
    float2* O = a.out + f * M;
    const float nrm = a.norm;
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
        const int k2 = (ka + 16 * kb + 128) & 255;
        const float2 y = make_float2(v[kb].x * nrm, v[kb].y * nrm);
        if (NT) st_nt(O + (long)k2 * 256 + k1b + r, y);
        else O[(long)k2 * 256 + k1b + r] = y;
    }
}


// -------- one-pass radix-4 DIF for N = 4M, 8192 <= N <= 65536 (configs[2]'s 64 Ki frames) --
// X[4k + m] = DFT_M(y_m)[k],  y_m[n] = (sum_p q_p[n] (-i)^{pm}) W_N^{mn},  q_p[n] = x[n + pM].
// Workgroup (frame, m) computes one M-point transform (M <= 16384: 136 KiB padded LDS tile,
// 1024 lanes x 16 points), reading the whole frame to form y_m in its load and writing every
// 4th output bin.  No scratch slab and no inter-workgroup exchange: the four workgroups of a
// frame share its input lines (and consecutive frames their overlap) through the XCD's L2,
// and their interleaved plain stores merge into whole lines there before write-back.  Blocks
// b, b+8, b+16, b+24 take the four m of one frame and each block group b % 8 a contiguous
// range of frames -- on the round-robin XCD placement that keeps a frame (and its neighbours)
// on one XCD (speed only; any placement gives the same results).
struct Dif4Args {
    FrameSrc src;
    long nframes;
    long fpg;           // frames per block group (ceil(nframes / 8))
    const float2* twN;  // W_N, N entries
    float norm;
    int store_mode;
    float2* out;
};

template <int R, int M, int NS, int NTH>
__device__ __forceinline__ void dif4_pass(float2* lds, const float2* __restrict__ twN) {
    constexpr int NBF = 16 / R;
    constexpr int BPT = M / R;
    const int t = threadIdx.x;
    float2 v[NBF][R];
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
        const int j = t * NBF + u;
#pragma unroll
        for (int r = 0; r < R; ++r) v[u][r] = lds[fpad(j + r * BPT)];
        if (NS > 1) {
            const int k = j % NS;
            twiddle<R, false>(v[u], twN, 4 * k * (M / (NS * R)));  // W_M^k = W_N^{4k}
        }
        Dft<R, false>::run(v[u]);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
        const int j = t * NBF + u;
        const int k = j % NS;
        const int o = (j / NS) * NS * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) lds[fpad(o + r * NS)] = v[u][r];
    }
    __syncthreads();
}

template <int M, int NS, int NTH>
__device__ __forceinline__ void dif4_fft(float2* lds, const float2* __restrict__ twN) {
    if constexpr (NS < M) {
        constexpr int LEFT = M / NS;
        constexpr int R = LEFT >= 16 ? 16 : LEFT;
        dif4_pass<R, M, NS, NTH>(lds, twN);
        dif4_fft<M, NS * R, NTH>(lds, twN);
    }
}

template <int M>
__global__ __launch_bounds__(M / 16) void fft_dif4_kernel(Dif4Args a) {
    constexpr int NTH = M / 16;
    constexpr long N = 4L * M;
    extern __shared__ float2 dlds[];
    const int t = threadIdx.x;
    const long b = blockIdx.x;
    const long g = b & 7, i = b >> 3;
    const int m = (int)(i & 3);
    const long f = g * a.fpg + (i >> 2);
    if (f >= a.nframes) return;
    const FrameSrc& s = a.src;
    const float2* base = nullptr;  // fast path: the whole frame is contiguous in memory
    if (s.mode == 0) base = s.in + f * N;
    else if (s.mode == 1) {
        const long g0 = s.first_end + f * s.hop - N;
        if (g0 >= 0 && g0 + N <= s.n_in) base = s.in + g0;
    }
    // load + first radix-4 stage (output m only) + W_N^{mn}
#pragma unroll 8
    for (int q = 0; q < 16; ++q) {
        const int n = t + NTH * q;
        float2 x0, x1, x2, x3;
        if (base) {
            x0 = base[n];
            x1 = base[n + M];
            x2 = base[n + 2 * M];
            x3 = base[n + 3 * M];
        } else {
            x0 = frame_sample(s, N, f, n);
            x1 = frame_sample(s, N, f, n + M);
            x2 = frame_sample(s, N, f, n + 2 * M);
            x3 = frame_sample(s, N, f, n + 3 * M);
        }
        dft4<false>(x0, x1, x2, x3);
        float2 y = m == 0 ? x0 : (m == 1 ? x1 : (m == 2 ? x2 : x3));
        if (m) y = cmul(y, a.twN[m * n]);
        dlds[fpad(n)] = y;
    }
    __syncthreads();
    dif4_fft<M, 1, NTH>(dlds, a.twN);
    // bin 4k + m of frame f
    if (a.store_mode == 0) {
        float2* O = a.out + f * N;
#pragma unroll 4
        for (int q = 0; q < 16; ++q) {
            const int k = t + NTH * q;
            const float2 x = dlds[fpad(k)];
            const long o = (4L * k + m + N / 2) & (N - 1);
            O[o] = make_float2(x.x * a.norm, x.y * a.norm);
        }
    } else {
#pragma unroll 4
        for (int q = 0; q < 16; ++q) {
            const int k = t + NTH * q;
            store_bin(a.out, f, N, 4L * k + m, dlds[fpad(k)], a.store_mode, a.norm);
        }
    }
}

}  // namespace

// ------------------------------ plan / launch -------------------------------------------
struct FftPlanDev {
    int M = 0;
    int M1 = 0, M2 = 0;
    float norm = 1.f;
    float2* tw4096 = nullptr;
    float2* twM = nullptr;
    // 64K four-step, two-stream mode: batches alternate between the caller's stream and
    // `aux` (each with its own half of the scratch slab) so one batch's pass B overlaps the
    // next batch's pass A instead of draining the GPU at every pass boundary
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    void* gen = nullptr;  // sizes that are not powers of two (fft_gen.hip)
};

void* fft_plan_create(int M, int* status) {
    if (M < 1 || M > (1 << 24)) {
        *status = SDRGPU_ERR_UNSUPPORTED;
        return nullptr;
    }
    if (M == 1 || (M & (M - 1))) {
        void* g = fftgen_plan_create(M, status);
        if (!g) return nullptr;
        auto* p = new FftPlanDev();
        p->M = M;
        p->gen = g;
        return p;
    }
    if (M > (1 << 20)) {
        *status = SDRGPU_ERR_UNSUPPORTED;
        return nullptr;
    }
    auto* p = new FftPlanDev();
    p->M = M;
    p->norm = 1.0f / sqrtf((float)M);  // f32, like fft.rs:16
    std::vector<float2> tw(kTile);
    for (int m = 0; m < kTile; ++m) {
        const double ang = -2.0 * M_PI * (double)m / kTile;
        tw[m] = make_float2((float)std::cos(ang), (float)std::sin(ang));
    }
    bool ok = hipMalloc(&p->tw4096, kTile * sizeof(float2)) == hipSuccess &&
              hipMemcpy(p->tw4096, tw.data(), kTile * sizeof(float2), hipMemcpyHostToDevice) == hipSuccess;
    if (ok && M > kTile) {
        // M = M1 * M2 with M2 = largest power of two <= sqrt(M) bounded by the tile
        int l2 = 0;
        while ((1 << l2) < M) ++l2;
        p->M2 = 1 << (l2 / 2);
        p->M1 = M / p->M2;
        std::vector<float2> twm(M);
        for (int m = 0; m < M; ++m) {
            const double ang = -2.0 * M_PI * (double)m / M;
            twm[m] = make_float2((float)std::cos(ang), (float)std::sin(ang));
        }
        ok = hipMalloc(&p->twM, (size_t)M * sizeof(float2)) == hipSuccess &&
             hipMemcpy(p->twM, twm.data(), (size_t)M * sizeof(float2), hipMemcpyHostToDevice) == hipSuccess;
    }
    if (!ok) {
        fft_plan_destroy(p);
        *status = SDRGPU_ERR_NOMEM;
        return nullptr;
    }
    *status = SDRGPU_OK;
    return p;
}

void fft_plan_destroy(void* plan) {
    auto* p = static_cast<FftPlanDev*>(plan);
    if (!p) return;
    if (p->gen) fftgen_plan_destroy(p->gen);
    if (p->tw4096) (void)hipFree(p->tw4096);
    if (p->twM) (void)hipFree(p->twM);
    if (p->aux) (void)hipStreamSynchronize(p->aux);
    if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
    if (p->ev_join) (void)hipEventDestroy(p->ev_join);
    if (p->aux) (void)hipStreamDestroy(p->aux);
    delete p;
}

int fft_plan_size(void* plan) { return static_cast<FftPlanDev*>(plan)->M; }

// one-pass radix-4 DIF sizes (no scratch slab): 8192 <= M <= 32768.  Measured for STFTs at
// hop N/2 over 2^28 samples (profiles/r02_stft_dif4_ab.txt): 3.0-3.7 ms against 5.3-5.6 ms for
// the generic four-step; at 65536 the one-pass form is latency-bound (one 139 KiB workgroup
// per CU, phases serialised: 4.1 ms) and the dedicated 64K two-pass path below wins (2.2 ms).
static bool use_dif4(int M) { return M >= 8192 && M <= 32768; }

static size_t frame_scratch_bytes(const FftPlanDev* p) {
    if (p->gen) return fftgen_frame_scratch_bytes(p->gen);
    return (p->M <= kTile || use_dif4(p->M)) ? 0 : (size_t)p->M * sizeof(float2);
}

template <int MQ>
static int launch_dif4(const FftPlanDev* p, const FrameSrc& src, long nframes, float2* out,
                       int store_mode, hipStream_t s) {
    constexpr size_t lds = (size_t)(MQ + MQ / 16) * sizeof(float2);
    static const bool attr = hipFuncSetAttribute((const void*)fft_dif4_kernel<MQ>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lds) == hipSuccess;
    if (!attr) return SDRGPU_ERR_LAUNCH;
    Dif4Args a{};
    a.src = src;
    a.nframes = nframes;
    a.fpg = (nframes + 7) / 8;
    a.twN = p->twM;
    a.norm = p->norm;
    a.store_mode = store_mode;
    a.out = out;
    hipLaunchKernelGGL(fft_dif4_kernel<MQ>, dim3((unsigned)(32 * a.fpg)), dim3(MQ / 16), lds, s, a);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

size_t fft_scratch_bytes(void* plan) {
    return fft_scratch_frames(plan) * frame_scratch_bytes(static_cast<FftPlanDev*>(plan));
}

size_t fft_scratch_frames(void* plan) {
    auto* p = static_cast<FftPlanDev*>(plan);
    const size_t per = frame_scratch_bytes(p);
    if (per == 0) return 0;
    // scratch slab of 256 MiB (the MALL size): 512 workgroups per pass, 32 launches per 2^28
    // samples; measured 2.79 ms vs 2.92 (128 MiB), 3.08 (64 MiB), 3.23 (512 MiB)
    // (profiles/r01_fft64k_experiments.txt)
    constexpr size_t kSlabBytes = (size_t)256 << 20;
    return std::max<size_t>(1, kSlabBytes / per);
}

int fft_launch(void* plan, const FftFrames& fr, float2* out, int store_mode, float2* scratch,
               size_t scratch_frames, hipStream_t s) {
    auto* p = static_cast<FftPlanDev*>(plan);
    if (p->gen) return fftgen_launch(p->gen, fr, out, store_mode, scratch, scratch_frames, s);
    FrameSrc src;
    src.mode = fr.mode;
    src.in = fr.in;
    src.in_real = fr.in_real;
    src.in_u8 = fr.in_u8;
    src.n_in = fr.n_in;
    src.hist = fr.hist;
    src.H = fr.H;
    src.first_end = fr.first_end;
    src.hop = fr.hop;
    if (fr.nframes <= 0) return SDRGPU_OK;
    if (p->M <= kTile) {
        TileArgs a{};
        a.src = src;
        a.nframes = fr.nframes;
        a.M = p->M;
        a.tw = p->tw4096;
        a.norm = p->norm;
        a.store_mode = store_mode;
        a.out = out;
        const long fpt = kTile / p->M;
        const dim3 g((unsigned)((fr.nframes + fpt - 1) / fpt)), b(kFftBlock);
        switch (p->M) {
        case 2: hipLaunchKernelGGL(fft_tile_kernel<2>, g, b, 0, s, a); break;
        case 4: hipLaunchKernelGGL(fft_tile_kernel<4>, g, b, 0, s, a); break;
        case 8: hipLaunchKernelGGL(fft_tile_kernel<8>, g, b, 0, s, a); break;
        case 16: hipLaunchKernelGGL(fft_tile_kernel<16>, g, b, 0, s, a); break;
        case 32: hipLaunchKernelGGL(fft_tile_kernel<32>, g, b, 0, s, a); break;
        case 64: hipLaunchKernelGGL(fft_tile_kernel<64>, g, b, 0, s, a); break;
        case 128: hipLaunchKernelGGL(fft_tile_kernel<128>, g, b, 0, s, a); break;
        case 256: hipLaunchKernelGGL(fft_tile_kernel<256>, g, b, 0, s, a); break;
        case 512: hipLaunchKernelGGL(fft_tile_kernel<512>, g, b, 0, s, a); break;
        case 1024: hipLaunchKernelGGL(fft_tile_kernel<1024>, g, b, 0, s, a); break;
        case 2048: hipLaunchKernelGGL(fft_tile_kernel<2048>, g, b, 0, s, a); break;
        case 4096: hipLaunchKernelGGL(fft_tile_kernel<4096>, g, b, 0, s, a); break;
        default: return SDRGPU_ERR_UNSUPPORTED;
        }
        SDRGPU_LAUNCH_CHECK();
        return SDRGPU_OK;
    }
    if (use_dif4(p->M)) {
        switch (p->M) {
        case 8192: return launch_dif4<2048>(p, src, fr.nframes, out, store_mode, s);
        case 16384: return launch_dif4<4096>(p, src, fr.nframes, out, store_mode, s);
        default: return launch_dif4<8192>(p, src, fr.nframes, out, store_mode, s);
        }
    }
    if (!scratch || scratch_frames == 0) return SDRGPU_ERR_UNSUPPORTED;
    if (p->M == 65536) {
        // 32 columns per workgroup (CB = 64: 3.36 vs 2.94 ms), non-temporal stream loads and
        // stores (2.92 vs 3.01 ms), two streams once there is more than half a slab of frames
        // (2.63-2.70 vs 2.77-2.79 ms): profiles/r01_fft64k_experiments.txt
        constexpr int cb = 32;
        const bool two = scratch_frames >= 2 && fr.nframes > (long)scratch_frames / 2;
        if (two && !p->aux) {
            if (hipStreamCreateWithFlags(&p->aux, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming) != hipSuccess)
                return SDRGPU_ERR_DEVICE;
        }
        const long batch = two ? (long)scratch_frames / 2 : (long)scratch_frames;
        if (two) {  // aux starts after everything already queued on s
            if (hipEventRecord(p->ev_fork, s) != hipSuccess ||
                hipStreamWaitEvent(p->aux, p->ev_fork, 0) != hipSuccess)
                return SDRGPU_ERR_DEVICE;
        }
        F64Args a{};
        a.tw = p->tw4096;
        a.twM = p->twM;
        a.norm = p->norm;
        a.store_mode = store_mode;
        long bi = 0;
        for (long f0 = 0; f0 < fr.nframes; f0 += batch, ++bi) {
            const long nf = std::min(batch, fr.nframes - f0);
            const bool odd = two && (bi & 1);
            hipStream_t st = odd ? p->aux : s;
            a.scratch = scratch + (odd ? batch * (long)p->M : 0L);
            a.src = src;
            if (frame_src_is_stream(src.mode)) a.src.first_end = src.first_end + f0 * src.hop;
            else if (src.mode == 0) a.src.in = src.in + f0 * (long)p->M;
            else a.src.in_real = src.in_real + f0 * (long)p->M;
            a.nframes = nf;
            a.out = store_advance(out, f0, p->M, store_mode);
            const dim3 g((unsigned)(nf * (256 / cb))), b(16 * cb);
            hipLaunchKernelGGL((fft64k_pass_a<cb, true>), g, b, 0, st, a);
            SDRGPU_LAUNCH_CHECK();
            hipLaunchKernelGGL((fft64k_pass_b<cb, true>), g, b, 0, st, a);
            SDRGPU_LAUNCH_CHECK();
        }
        if (two) {  // s continues only after aux's batches
            if (hipEventRecord(p->ev_join, p->aux) != hipSuccess ||
                hipStreamWaitEvent(s, p->ev_join, 0) != hipSuccess)
                return SDRGPU_ERR_DEVICE;
        }
        return SDRGPU_OK;
    }
    FourArgs a{};
    a.M = p->M;
    a.M1 = p->M1;
    a.M2 = p->M2;
    a.tw = p->tw4096;
    a.twM = p->twM;
    a.norm = p->norm;
    a.store_mode = store_mode;
    a.scratch = scratch;
    for (long f0 = 0; f0 < fr.nframes; f0 += (long)scratch_frames) {
        const long nf = std::min((long)scratch_frames, fr.nframes - f0);
        a.src = src;
        if (frame_src_is_stream(src.mode)) a.src.first_end = src.first_end + f0 * src.hop;
        else if (src.mode == 0) a.src.in = src.in + f0 * (long)p->M;
        else a.src.in_real = src.in_real + f0 * (long)p->M;
        a.nframes = nf;
        a.out = store_advance(out, f0, p->M, store_mode);
        const long ga = nf * (a.M1 / (kTile / a.M2));
        const long gb = nf * (a.M2 / (kTile / a.M1));
        const dim3 bA((unsigned)ga), bB((unsigned)gb), b(kFftBlock);
        switch (a.M2) {
        case 64: hipLaunchKernelGGL(fft4_pass_a<64>, bA, b, 0, s, a); break;
        case 128: hipLaunchKernelGGL(fft4_pass_a<128>, bA, b, 0, s, a); break;
        case 256: hipLaunchKernelGGL(fft4_pass_a<256>, bA, b, 0, s, a); break;
        case 512: hipLaunchKernelGGL(fft4_pass_a<512>, bA, b, 0, s, a); break;
        case 1024: hipLaunchKernelGGL(fft4_pass_a<1024>, bA, b, 0, s, a); break;
        default: return SDRGPU_ERR_UNSUPPORTED;
        }
        SDRGPU_LAUNCH_CHECK();
        switch (a.M1) {
        case 128: hipLaunchKernelGGL(fft4_pass_b<128>, bB, b, 0, s, a); break;
        case 256: hipLaunchKernelGGL(fft4_pass_b<256>, bB, b, 0, s, a); break;
        case 512: hipLaunchKernelGGL(fft4_pass_b<512>, bB, b, 0, s, a); break;
        case 1024: hipLaunchKernelGGL(fft4_pass_b<1024>, bB, b, 0, s, a); break;
        default: return SDRGPU_ERR_UNSUPPORTED;
        }
        SDRGPU_LAUNCH_CHECK();
    }
    return SDRGPU_OK;
}

// history carry for the STFT stream: hist_next[j] = stream sample (n_in - H + j)
__global__ void stft_carry_kernel(const float2* in, long n_in, const float2* hist, float2* hist_next,
                                  long H) {
    for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < H; j += (long)gridDim.x * blockDim.x) {
        const long g = n_in - H + j;
        hist_next[j] = g >= 0 ? in[g] : hist[g + H];
    }
}

__global__ void stft_carry_u8_kernel(const unsigned short* in, long n_in, const float2* hist,
                                     float2* hist_next, long H) {
    for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < H; j += (long)gridDim.x * blockDim.x) {
        const long g = n_in - H + j;
        hist_next[j] = g >= 0 ? u8_sample(in[g]) : hist[g + H];
    }
}

int stft_carry_u8_launch(const unsigned short* in, long n_in, const float2* hist,
                         float2* hist_next, long H, hipStream_t s) {
    if (H <= 0) return SDRGPU_OK;
    const long nb = std::min<long>((H + 255) / 256, 1024);
    hipLaunchKernelGGL(stft_carry_u8_kernel, dim3((unsigned)nb), dim3(256), 0, s, in, n_in, hist,
                       hist_next, H);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

int stft_carry_launch(const float2* in, long n_in, const float2* hist, float2* hist_next, long H,
                      hipStream_t s) {
    if (H <= 0) return SDRGPU_OK;
    const long nb = std::min<long>((H + 255) / 256, 1024);
    hipLaunchKernelGGL(stft_carry_kernel, dim3((unsigned)nb), dim3(256), 0, s, in, n_in, hist, hist_next, H);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

}  // namespace sdrgpu
