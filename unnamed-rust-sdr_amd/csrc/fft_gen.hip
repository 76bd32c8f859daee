// fft_gen.hip -- fft::fft / fft::rfft / STFT for sizes that are not powers of two (gfx950).
//
// rustfft plans any length (reference src/fft.rs:10-11; FFTplanner::new(false) = forward),
// and the reference's own callers use such lengths: examples/live.rs:30 frames a 1000-point
// window (window(1000 / rate)) and examples/fft.rs:64,78 rffts take(0.1) of a 144 kHz
// stream = 14,400 points.  Output semantics are those of fft.hip (collated, x 1/sqrt(N) in
// f32, fft.rs:14-26; rfft keeps collated [N/2, N), fft.rs:35).
//
// Three plans, chosen on the host from N's factorisation:
//   * mixed-radix tile (N <= 4096, every prime factor <= 13): B = 4096/N transforms per
//     256-lane workgroup in one 32 KiB LDS buffer, one in-place Stockham autosort
//     pass per radix (16/8/4/2, 3, 5, and a generic odd-radix pair kernel for 7/11/13);
//     twiddles: one load per butterfly from a W_N table computed in f64 on the host, its
//     powers by a log-depth product tree; index arithmetic by plan-time magic multipliers;
//     the STFT frame gather and the collated store are folded into the first / last pass.
//   * mixed-radix four-step (N > 4096 smooth, N = N1 * N2 with both <= 4096):
//     pass A = N2-point FFTs down the columns n1 of x[n1 + N1 n2] (rows of C contiguous
//     samples), x W_N^{n1 k2}, to a scratch slab; pass B = N1-point FFTs over n1 for C'
//     consecutive k2, stored collated.  Both passes reuse the tile engine.
//   * Bluestein (a prime factor > 13): X[k] = w[k] sum_n (x[n] w[n]) conj(w[k - n]) with the
//     chirp w[n] = e^{-i pi n^2 / N} (n^2 mod 2N exact in integers, angle in f64); the
//     convolution runs as two power-of-two forward FFTs of size M >= 2N - 1 through the
//     fft.hip kernels (natural-order store) with the chirp spectrum conj(FFT_M(b)) / M
//     precomputed on the host in f64 (the second transform applies the inverse by
//     conjugation: IFFT(C) = conj(FFT(conj C)) / M).
// These are HBM-light, arithmetic-light transforms (no BASELINE config uses them); the
// power-of-two sizes (configs[2]'s 64 Ki STFT) never come here.
#include <algorithm>
#include <cmath>
#include <complex>
#include <vector>

#include "fft_device.hpp"
#include "fft_frames.hpp"
#include "fft_kernels.hpp"

namespace sdrgpu {

using namespace fftd;

namespace {

constexpr int kGenBlock = 256;
constexpr int kGenTile = 4096;   // complex points per LDS buffer
constexpr int kGenTileW = 1024;  // one-wave tiles (N <= 1024)
constexpr int kGenTileL = 16384; // one frame per 1024-lane workgroup, <= 128 KiB of LDS
constexpr int kGenBlockL = 1024;
#ifndef RFFT_BLK
#define RFFT_BLK 1024
#define RFFT_TILE 8192  // one frame per 1024-lane workgroup: 0.18 ms vs 0.25 (two frames), 0.20 (512 lanes)
#endif
constexpr int kRfftBlk = RFFT_BLK, kRfftTile = RFFT_TILE;  // packed 14,400-point rfft
#ifndef LIVE_BLK
#define LIVE_BLK 256  // 4 waves over 2 frames: 0.42 ms vs 0.46-0.47 (one wave per frame), 0.48 (128 lanes)
#define LIVE_TILE 2048
#endif
constexpr int kLiveBlk = LIVE_BLK, kLiveTile = LIVE_TILE;  // 1000-point live spectrum
constexpr int kMaxPass = 16;

// division by a plan-time constant d < 2^16 for dividends < 2^16: q = umulhi(n, ceil(2^32/d))
// (exact while n d < 2^32), one v_mul_hi_u32 instead of a ~30-instruction integer division
struct FastDiv {
    unsigned m = 0;
    int d = 1;
    __host__ void set(int dv) {
        d = dv;
        m = dv > 1 ? (unsigned)((0x100000000ULL + (unsigned long long)dv - 1) / (unsigned long long)dv) : 0u;
    }
    __device__ __forceinline__ int div(int n) const {
        return d == 1 ? n : (int)__umulhi((unsigned)n, m);
    }
};

struct RadixList {
    int n = 0;
    int R[kMaxPass] = {};
    FastDiv dq[kMaxPass];   // pass p: N / R[p] (butterflies per transform)
    FastDiv dns[kMaxPass];  // pass p: Ns = product of the earlier radices
    FastDiv dn;             // N
};

// LDS index of tile point i: one float2 of padding per 32, so the stride-R writes of a
// Stockham pass (R = 8, 16: 16- to 32-way bank conflicts unpadded) spread over the banks
// (the 16K-point single-frame tile only: at <= 4096 points the extra index arithmetic and
// the lost workgroup per CU cost more than the conflicts, profiles/r02_fft_anyn.txt)
template <int TILE>
__host__ __device__ __forceinline__ int lp(int i) { return TILE > 4096 ? i + (i >> 5) : i; }
template <int TILE>
__host__ inline size_t lp_bytes(int points) { return (size_t)lp<TILE>(points) * sizeof(float2) + sizeof(float2); }

// ---- butterflies -----------------------------------------------------------------------
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 cfma(float s, float2 a, float2 acc) {
    return make_float2(fmaf(s, a.x, acc.x), fmaf(s, a.y, acc.y));
}
// a - i b and a + i b
__device__ __forceinline__ float2 sub_i(float2 a, float2 b) { return make_float2(a.x + b.y, a.y - b.x); }
__device__ __forceinline__ float2 add_i(float2 a, float2 b) { return make_float2(a.x - b.y, a.y + b.x); }

__device__ __forceinline__ void dft3(float2* v) {
    constexpr float s = 0.86602540378443865f;  // sin(2 pi / 3)
    const float2 t1 = cadd(v[1], v[2]);
    const float2 t2 = make_float2(v[0].x - 0.5f * t1.x, v[0].y - 0.5f * t1.y);
    const float2 t3 = cscale(csub(v[1], v[2]), s);
    v[0] = cadd(v[0], t1);
    v[1] = sub_i(t2, t3);
    v[2] = add_i(t2, t3);
}

__device__ __forceinline__ void dft5(float2* v) {
    constexpr float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;
    constexpr float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;
    const float2 a1 = cadd(v[1], v[4]), a2 = cadd(v[2], v[3]);
    const float2 b1 = csub(v[1], v[4]), b2 = csub(v[2], v[3]);
    const float2 x0 = v[0];
    const float2 t1 = cfma(c2, a2, cfma(c1, a1, x0));
    const float2 t2 = cfma(c1, a2, cfma(c2, a1, x0));
    const float2 u1 = cfma(s2, b2, cscale(b1, s1));
    const float2 u2 = cfma(-s1, b2, cscale(b1, s2));
    v[0] = cadd(x0, cadd(a1, a2));
    v[1] = sub_i(t1, u1);
    v[4] = add_i(t1, u1);
    v[2] = sub_i(t2, u2);
    v[3] = add_i(t2, u2);
}

// any odd R: pairs a_m = x_m + x_{R-m}, b_m = x_m - x_{R-m};
// X_k = x0 + sum_m cos(2 pi mk/R) a_m - i sum_m sin(2 pi mk/R) b_m, X_{R-k} with + i.
// cos / sin come from the f64-accurate W_N table (R | N): W_N^{j N/R} = cos - i sin.
template <int R>
__device__ __forceinline__ void dft_odd(float2* v, const float2* __restrict__ tw, int N) {
    constexpr int H = (R - 1) / 2;
    const int st = N / R;
    float cs[R], sn[R];
#pragma unroll
    for (int j = 1; j < R; ++j) {
        const float2 w = tw[j * st];
        cs[j] = w.x;
        sn[j] = -w.y;
    }
    float2 a[H + 1], b[H + 1];
    float2 sum = v[0];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
        a[m] = cadd(v[m], v[R - m]);
        b[m] = csub(v[m], v[R - m]);
        sum = cadd(sum, a[m]);
    }
    const float2 x0 = v[0];
#pragma unroll
    for (int k = 1; k <= H; ++k) {
        float2 t = x0, u = make_float2(0.f, 0.f);
#pragma unroll
        for (int m = 1; m <= H; ++m) {
            const int j = (m * k) % R;
            t = cfma(cs[j], a[m], t);
            u = cfma(sn[j], b[m], u);
        }
        v[k] = sub_i(t, u);
        v[R - k] = add_i(t, u);
    }
    v[0] = sum;
}

template <int R>
__device__ __forceinline__ void dft_any(float2* v, const float2* __restrict__ tw, int N) {
    if constexpr (R == 2 || R == 4 || R == 8 || R == 16) Dft<R, false>::run(v);
    else if constexpr (R == 3) dft3(v);
    else if constexpr (R == 5) dft5(v);
    else dft_odd<R>(v, tw, N);
}

// One Stockham autosort pass over B transforms of size N (transform f at f * N), in place:
// every lane first reads and transforms its butterflies (f, j), j < N/R, k = j mod Ns
// (reads buf[f N + j + r N/R], twiddles by W_N^{r k N/(Ns R)}, a plain table index), then,
// after a barrier, writes them to buf[f N + (j - k) R + k + r Ns].  One LDS buffer instead of
// a ping-pong pair doubles the workgroups per CU.  B N <= 4096, so a lane owns at most
// ceil(4096 / (R 256)) butterflies.
template <int R, int BLK, int TILE>
__device__ __forceinline__ void gen_pass(float2* buf, int N, int B, int Ns,
                                         const float2* __restrict__ tw, const FastDiv& dq,
                                         const FastDiv& dns) {
    constexpr int NB = (TILE / R + BLK - 1) / BLK;
    const int Q = N / R;
    const int total = B * Q;
    const int step = N / (Ns * R);
    float2 v[NB][R];
    int dsto[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int g = threadIdx.x + u * BLK;
        dsto[u] = -1;
        if (g < total) {
            const int f = dq.div(g), j = g - f * Q;
            const int k = j - Ns * dns.div(j);
            const int s0 = f * N + j;
#pragma unroll
            for (int r = 0; r < R; ++r) v[u][r] = buf[lp<TILE>(s0 + r * Q)];
            if (Ns > 1) twiddle_tree<R>(v[u], tw[k * step]);  // W^{r k step} = (W^{k step})^r
            dft_any<R>(v[u], tw, N);
            dsto[u] = f * N + (j - k) * R + k;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        if (dsto[u] >= 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) buf[lp<TILE>(dsto[u] + r * Ns)] = v[u][r];
        }
    }
}

// Runs the plan's passes in place over B transforms of size N held in buf (BLK lanes, at
// most TILE points).
template <int BLK, int TILE>
__device__ void gen_engine(float2* buf, int N, int B, const RadixList& rl,
                           const float2* __restrict__ tw) {
    int Ns = 1;
    for (int ps = 0; ps < rl.n; ++ps) {
        const int R = rl.R[ps];
        const FastDiv& dq = rl.dq[ps];
        const FastDiv& dns = rl.dns[ps];
        switch (R) {
        case 2: gen_pass<2, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 3: gen_pass<3, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 4: gen_pass<4, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 5: gen_pass<5, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 7: gen_pass<7, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 8: gen_pass<8, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 11: gen_pass<11, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        case 13: gen_pass<13, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        default: gen_pass<16, BLK, TILE>(buf, N, B, Ns, tw, dq, dns); break;
        }
        __syncthreads();
        Ns *= R;
    }
}

struct GenTileArgs {
    FrameSrc src;
    long nframes;
    int N, B;
    RadixList rl;
    const float2* tw;  // W_N, N entries
    float norm;
    int store_mode;
    float2* out;
};

// BLK lanes over B = TILE / N frames: 256 lanes / 4096 points, or for N <= 1024 one wave
// over 1024 points (the passes' barriers are then single-wave; 8 KiB of LDS per wave)
template <int BLK, int TILE>
__global__ __launch_bounds__(BLK) void gen_tile_kernel(GenTileArgs a) {
    extern __shared__ float2 glds[];
    const int N = a.N, B = a.B, L = B * N;
    float2* b0 = glds;
    const long f0 = (long)blockIdx.x * B;
    const int nf = (int)min((long)B, a.nframes - f0);
    {  // every lane's loads in flight before the first LDS write (unrolled, predicated)
        constexpr int PER = TILE / BLK;
        float2 v[PER];
        gather_tile<PER, BLK>(a.src, N, f0, nf, L, [&](int p) { return a.rl.dn.div(p); }, v);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * BLK;
            if (p < L) b0[lp<TILE>(p)] = v[u];
        }
    }
    __syncthreads();
    gen_engine<BLK, TILE>(b0, N, B, a.rl, a.tw);
    const float2* X = b0;
    if (a.store_mode == 0 || a.store_mode == 3) {
        // output-ordered: out[o] = X[(o - N/2) mod N] * norm, consecutive lanes -> consecutive o;
        // the dB store writes output (f, o) as element p = f N + o of the workgroup's contiguous
        // output run, a 32-bit offset off one scalar base (the c64 store the same way measured
        // 1-2 % slower at 1200 / 6000 points, faster at 3000: not taken, profiles/r06_fftfixed.txt)
        const int sh = N - N / 2;
        const bool db = a.store_mode == 3;
        char* base = reinterpret_cast<char*>(a.out) + f0 * N * 4;
        if (db) {
#pragma unroll 4
            for (int p = threadIdx.x; p < nf * N; p += BLK) {
                const int f = a.rl.dn.div(p), o = p - f * N;
                const float2 x = X[lp<TILE>(o + sh < N ? p + sh : p + sh - N)];
                *reinterpret_cast<float*>(base + (unsigned)p * 4u) = db_of(x, a.norm);
            }
        } else {
#pragma unroll 4
            for (int p = threadIdx.x; p < nf * N; p += BLK) {
                const int f = a.rl.dn.div(p), o = p - f * N;
                int k = o + sh;
                if (k >= N) k -= N;
                const float2 x = X[lp<TILE>(f * N + k)];
                a.out[(f0 + f) * N + o] = make_float2(x.x * a.norm, x.y * a.norm);
            }
        }
    } else {
        for (int p = threadIdx.x; p < nf * N; p += BLK) {
            const int f = a.rl.dn.div(p), k = p - f * N;
            store_bin(a.out, f0 + f, N, k, X[lp<TILE>(p)], a.store_mode, a.norm);
        }
    }
}

// ---- compile-time plans for the reference examples' sizes -------------------------------
// examples/live.rs frames 1000 points (window(1000 / rate)) and examples/fft.rs rffts 14,400
// (take(0.1) at 144 kHz); with N, the radix order and every
// stride known at compile time, the engine's index arithmetic (plan-time divisions, the pass
// loop's radix switch, the butterfly-count guards) folds into constants: the 1000-point live
// spectrum is VALU-bound (~2,700 VALU instructions per frame in the generic engine).  Same
// plan, twiddle table, pass order and arithmetic as gen_pass, so the results are identical.
template <int R, int BLK, int TILE, int N, int B, int NS>
__device__ __forceinline__ void fixed_pass(float2* buf, const float2* __restrict__ tw) {
    constexpr int Q = N / R, TOTAL = B * Q, STEP = N / (NS * R);
    constexpr int NB = (TOTAL + BLK - 1) / BLK;
    float2 v[NB][R];
    int dsto[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int g = threadIdx.x + u * BLK;
        dsto[u] = -1;
        if ((u + 1) * BLK <= TOTAL || g < TOTAL) {
            const int f = g / Q, j = g - f * Q;
            const int k = j % NS;
            const int s0 = f * N + j;
#pragma unroll
            for (int r = 0; r < R; ++r) v[u][r] = buf[lp<TILE>(s0 + r * Q)];
            // (the R - 1 powers read from the table instead: 1000 points 0.42 -> 0.55 ms, the
            // loads' latency costs more than the product tree's VALU, profiles/r06_fftfixed.txt)
            if (NS > 1) twiddle_tree<R>(v[u], tw[k * STEP]);
            dft_any<R>(v[u], tw, N);
            dsto[u] = f * N + (j - k) * R + k;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        if (dsto[u] >= 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) buf[lp<TILE>(dsto[u] + r * NS)] = v[u][r];
        }
    }
}

template <int BLK, int TILE, int N, int B, int NS, int R, int... REST>
__device__ __forceinline__ void fixed_engine(float2* buf, const float2* __restrict__ tw) {
    fixed_pass<R, BLK, TILE, N, B, NS>(buf, tw);
    __syncthreads();
    if constexpr (sizeof...(REST) > 0) fixed_engine<BLK, TILE, N, B, NS * R, REST...>(buf, tw);
}

template <int BLK, int TILE, int N, int... RS>
__global__ __launch_bounds__(BLK) void gen_fixed_kernel(GenTileArgs a) {
    extern __shared__ float2 glds[];
    constexpr int B = TILE / N, L = B * N;
    float2* b0 = glds;
    const long f0 = (long)blockIdx.x * B;
    const int nf = (int)min((long)B, a.nframes - f0);
    {
        constexpr int PER = TILE / BLK;
        float2 v[PER];
        gather_tile_ct<PER, BLK, N, L>(a.src, f0, nf, v);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * BLK;
            if (p < L) b0[lp<TILE>(p)] = v[u];
        }
    }
    __syncthreads();
    fixed_engine<BLK, TILE, N, B, 1, RS...>(b0, a.tw);
    const float2* X = b0;
    if ((a.store_mode == 0 || a.store_mode == 3) && nf == B) {
        // full workgroup: output element (f, o) is element p = f N + o of the workgroup's
        // contiguous output run, a 32-bit offset off one scalar base
        constexpr int SH = N - N / 2, NU = (L + BLK - 1) / BLK;
        const bool db = a.store_mode == 3;
        char* base = reinterpret_cast<char*>(a.out) + f0 * N * (db ? 4 : 8);
        float2 x[NU];  // every LDS read issued before the first store
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int p = threadIdx.x + u * BLK, f = p / N, o = p - f * N;
            x[u] = p < L ? X[lp<TILE>(o + SH < N ? p + SH : p + SH - N)] : make_float2(0.f, 0.f);
        }
        if (db) {
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int p = threadIdx.x + u * BLK;
                if (p < L) *reinterpret_cast<float*>(base + (unsigned)p * 4u) = db_of(x[u], a.norm);
            }
        } else {
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int p = threadIdx.x + u * BLK;
                if (p < L)
                    *reinterpret_cast<float2*>(base + (unsigned)p * 8u) = make_float2(x[u].x * a.norm, x[u].y * a.norm);
            }
        }
    } else if (a.store_mode == 0 || a.store_mode == 3) {
        constexpr int SH = N - N / 2;
#pragma unroll
        for (int u = 0; u < (L + BLK - 1) / BLK; ++u) {
            const int p = threadIdx.x + u * BLK;
            const int f = p / N, o = p - f * N;
            if (p < L && f < nf) {
                const int k = o + SH < N ? o + SH : o + SH - N;
                const float2 x = X[lp<TILE>(f * N + k)];
                if (a.store_mode == 0) a.out[(f0 + f) * N + o] = make_float2(x.x * a.norm, x.y * a.norm);
                else reinterpret_cast<float*>(a.out)[(f0 + f) * N + o] = db_of(x, a.norm);
            }
        }
    } else {
        for (int p = threadIdx.x; p < nf * N; p += BLK) {
            const int f = p / N, k = p - f * N;
            store_bin(a.out, f0 + f, N, k, X[lp<TILE>(p)], a.store_mode, a.norm);
        }
    }
}

// examples/fft.rs's rfft at its size (real 14,400-point frames, bins [0, N/2) of the collated
// output, fft.rs:30-37) by the half-length packing: z[n] = x[2n] + i x[2n+1] is the real frame
// read as NH = N/2 complex points, Z = FFT_NH(z) in LDS (the same compile-time engine), then
// X[k] = (Z[k] + Z*[NH-k]) / 2 - i W_N^k (Z[k] - Z*[NH-k]) / 2 for the kept bins -- half the
// transform work of the zero-imaginary N-point transform, same 1/sqrt(N) scale.  Parity is
// the FFT's (1e-5 of RMS against the f64 DFT), not bit-equality with the full transform.
template <int BLK, int TILE, int NH, int... RS>
__global__ __launch_bounds__(BLK) void gen_rfft_half_kernel(GenTileArgs a, const float2* __restrict__ twh) {
    extern __shared__ float2 glds[];
    constexpr int B = TILE / NH, L = B * NH;
    float2* b0 = glds;
    const long f0 = (long)blockIdx.x * B;
    const int nf = (int)min((long)B, a.nframes - f0);
    {
        constexpr int PER = TILE / BLK;
        float2 v[PER];
        gather_tile_ct<PER, BLK, NH, L>(a.src, f0, nf, v);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * BLK;
            if (p < L) b0[lp<TILE>(p)] = v[u];
        }
    }
    __syncthreads();
    fixed_engine<BLK, TILE, NH, B, 1, RS...>(b0, twh);
    // bin (f, k) is element p = f NH + k of the workgroup's contiguous output run: a 32-bit
    // offset off one scalar base
    const bool db = a.store_mode != 1;
    char* base = reinterpret_cast<char*>(a.out) + f0 * NH * (db ? 4 : 8);
#pragma unroll 2  // (fully unrolled: 70 VGPRs, one workgroup per CU fewer)
    for (int u = 0; u < (L + BLK - 1) / BLK; ++u) {
        const int p = threadIdx.x + u * BLK;
        if (p < L && p < nf * NH) {
            const int f = p / NH, k = p - f * NH;
            const float2 z = b0[lp<TILE>(p)];
            const float2 m = b0[lp<TILE>(f * NH + (k ? NH - k : 0))];
            const float ex = 0.5f * (z.x + m.x), ey = 0.5f * (z.y - m.y);
            const float ox = 0.5f * (z.y + m.y), oy = -0.5f * (z.x - m.x);
            const float2 w = a.tw[k];  // W_N^k, N = 2 NH
            const float2 x = make_float2(ex + (w.x * ox - w.y * oy), ey + (w.x * oy + w.y * ox));
            if (!db) *reinterpret_cast<float2*>(base + (unsigned)p * 8u) = make_float2(x.x * a.norm, x.y * a.norm);
            else *reinterpret_cast<float*>(base + (unsigned)p * 4u) = db_of(x, a.norm);
        }
    }
}

// ---- four-step over two mixed-radix tiles (n = n1 + N1 n2, k = k2 + N2 k1) -------------
struct Gen4Args {
    FrameSrc src;
    long nframes;
    int N, N1, N2;
    RadixList rlA, rlB;      // N2-point (pass A) and N1-point (pass B) plans
    const float2* twA;       // W_N2
    const float2* twB;       // W_N1
    const float2* twN;       // W_N
    float norm;
    int store_mode;
    float2* scratch;         // nframes x N: S[f][n1 N2 + k2]
    float2* out;
};

// p / d for p, d <= 4096 with d varying per workgroup: f32 reciprocal estimate, then one
// correction step each way (exact: the estimate is off by at most one)
__device__ __forceinline__ int small_div(int p, int d) {
    int q = (int)((float)p * __builtin_amdgcn_rcpf((float)d));
    q += (q + 1) * d <= p;
    q -= q * d > p;
    return q;
}

__global__ __launch_bounds__(kGenBlock) void gen4_pass_a(Gen4Args a) {
    extern __shared__ float2 glds[];
    const int N1 = a.N1, N2 = a.N2;
    const int C = kGenTile / N2;
    const int tiles = (N1 + C - 1) / C;
    const long f = blockIdx.x / tiles;
    const int c0 = (int)(blockIdx.x % tiles) * C;
    if (f >= a.nframes) return;
    const int nc = min(C, N1 - c0);
    float2* b0 = glds;
    {  // rows of nc contiguous samples (lanes walk the column); all loads in flight first
        constexpr int PER = kGenTile / kGenBlock;
        float2 v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * kGenBlock;
            const int n2 = small_div(p, nc), col = p - n2 * nc;
            v[u] = p < nc * N2 ? frame_sample(a.src, a.N, f, (long)(c0 + col) + (long)N1 * n2)
                               : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * kGenBlock;
            const int n2 = small_div(p, nc), col = p - n2 * nc;
            if (p < nc * N2) b0[lp<kGenTile>(col * N2 + n2)] = v[u];
        }
    }
    __syncthreads();
    gen_engine<kGenBlock, kGenTile>(b0, N2, nc, a.rlA, a.twA);
    const float2* X = b0;
    float2* S = a.scratch + f * (long)a.N + (long)c0 * N2;
    for (int p = threadIdx.x; p < nc * N2; p += kGenBlock) {
        const int col = a.rlA.dn.div(p), k2 = p - col * N2;
        S[p] = cmul(X[lp<kGenTile>(p)], a.twN[(c0 + col) * k2]);   // (n1 k2 < N)
    }
}

__global__ __launch_bounds__(kGenBlock) void gen4_pass_b(Gen4Args a) {
    extern __shared__ float2 glds[];
    const int N1 = a.N1, N2 = a.N2;
    const int C = kGenTile / N1;
    const int tiles = (N2 + C - 1) / C;
    const long f = blockIdx.x / tiles;
    const int c0 = (int)(blockIdx.x % tiles) * C;
    if (f >= a.nframes) return;
    const int nc = min(C, N2 - c0);
    float2* b0 = glds;
    const float2* S = a.scratch + f * (long)a.N;
    {
        constexpr int PER = kGenTile / kGenBlock;
        float2 v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * kGenBlock;
            const int n1 = small_div(p, nc), col = p - n1 * nc;
            v[u] = p < nc * N1 ? S[(long)n1 * N2 + c0 + col] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = threadIdx.x + u * kGenBlock;
            const int n1 = small_div(p, nc), col = p - n1 * nc;
            if (p < nc * N1) b0[lp<kGenTile>(col * N1 + n1)] = v[u];
        }
    }
    __syncthreads();
    gen_engine<kGenBlock, kGenTile>(b0, N1, nc, a.rlB, a.twB);
    const float2* X = b0;
    for (int p = threadIdx.x; p < nc * N1; p += kGenBlock) {
        const int k1 = small_div(p, nc), col = p - k1 * nc;
        const long k = (long)(c0 + col) + (long)N2 * k1;
        store_bin(a.out, f, a.N, k, X[lp<kGenTile>(col * N1 + k1)], a.store_mode, a.norm);
    }
}

// ---- Bluestein --------------------------------------------------------------------------
struct BluArgs {
    FrameSrc src;
    long nframes;
    int N, M;
    const float2* chirp;  // w[n] = e^{-i pi n^2 / N}, N entries
    const float2* bhat;   // FFT_M(b) / M, see blu_mid
    float2* T;            // nframes x M work frames
    float2* U;            // a second nframes x M set (the power-of-two kernels run out of place)
    float norm;
    int store_mode;
    float2* out;
};

__global__ void blu_pre(BluArgs a) {
    const long total = a.nframes * (long)a.M;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const long f = i / a.M;
        const int m = (int)(i - f * a.M);
        a.T[i] = m < a.N ? cmul(frame_sample(a.src, a.N, f, m), a.chirp[m]) : make_float2(0.f, 0.f);
    }
}

// T = conj(U * Bh) with U = FFT(a) and Bh = FFT_M(b) / M: the next forward transform then
// gives conj(M * IFFT(FFT(a) Bh)) = conj(a (*) b) (circular convolution of length M)
__global__ void blu_mid(BluArgs a) {
    const long total = a.nframes * (long)a.M;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const int m = (int)(i % a.M);
        a.T[i] = conjf2(cmul(a.U[i], a.bhat[m]));
    }
}

__global__ void blu_post(BluArgs a) {
    const long total = a.nframes * (long)a.N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const long f = i / a.N;
        const int k = (int)(i - f * a.N);
        const float2 c = conjf2(a.U[f * a.M + k]);
        store_bin(a.out, f, a.N, k, cmul(a.chirp[k], c), a.store_mode, a.norm);
    }
}

// ---- host side ----------------------------------------------------------------------------
bool radices(int n, RadixList& rl) {
    rl.n = 0;
    int twos = 0;
    while (n % 2 == 0) {
        n /= 2;
        ++twos;
    }
    // odd radices first, the power-of-two radices last: a Stockham pass writes at stride R
    // while Ns = 1 and contiguously once Ns = N / R, so the 8 / 16 (bank-conflicting at
    // stride R) go where their writes are contiguous
    for (int p : {3, 5, 7, 11, 13}) {
        while (n % p == 0) {
            if (rl.n >= kMaxPass) return false;
            rl.R[rl.n++] = p;
            n /= p;
        }
    }
    if (n != 1) return false;
    if (twos % 4) rl.R[rl.n++] = 1 << (twos % 4);
    for (; twos >= 4; twos -= 4) {
        if (rl.n >= kMaxPass) return false;
        rl.R[rl.n++] = 16;
    }
    int N = 1, Ns = 1;
    for (int i = 0; i < rl.n; ++i) N *= rl.R[i];
    for (int i = 0; i < rl.n; ++i) {
        rl.dq[i].set(N / rl.R[i]);
        rl.dns[i].set(Ns);
        Ns *= rl.R[i];
    }
    rl.dn.set(N);
    return true;
}

std::vector<float2> twiddles(long n) {
    std::vector<float2> t((size_t)n);
    for (long m = 0; m < n; ++m) {
        const double ang = -2.0 * M_PI * (double)m / (double)n;
        t[(size_t)m] = make_float2((float)std::cos(ang), (float)std::sin(ang));
    }
    return t;
}

// in-place iterative radix-2 forward DFT in f64 (host, plan time only)
void host_fft(std::vector<std::complex<double>>& a) {
    const size_t n = a.size();
    for (size_t i = 1, j = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        const double ang = -2.0 * M_PI / (double)len;
        for (size_t i = 0; i < n; i += len)
            for (size_t k = 0; k < len / 2; ++k) {
                const std::complex<double> w(std::cos(ang * k), std::sin(ang * k));
                const auto u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
    }
}

template <typename T>
bool upload(T** d, const std::vector<T>& h) {
    return hipMalloc(d, h.size() * sizeof(T)) == hipSuccess &&
           hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
}

enum { kTileKind = 1, kFourKind = 2, kBluKind = 3 };

}  // namespace

struct GenFftPlan {
    int N = 0, kind = 0;
    float norm = 1.f;
    RadixList rl, rlA, rlB;
    int N1 = 0, N2 = 0;
    float2 *tw = nullptr, *twA = nullptr, *twB = nullptr;
    float2* tw_half = nullptr;  // W_{N/2} for the packed real transform (N = 14400 only)
    int M = 0;
    void* inner = nullptr;  // power-of-two plan of size M (Bluestein)
    float2 *chirp = nullptr, *bhat = nullptr;
};

void fftgen_plan_destroy(void* plan) {
    auto* p = static_cast<GenFftPlan*>(plan);
    if (!p) return;
    for (float2* q : {p->tw, p->twA, p->twB, p->tw_half, p->chirp, p->bhat})
        if (q) (void)hipFree(q);
    if (p->inner) fft_plan_destroy(p->inner);
    delete p;
}

void* fftgen_plan_create(int N, int* status) {
    auto* p = new GenFftPlan();
    p->N = N;
    p->norm = 1.0f / sqrtf((float)N);  // f32, like fft.rs:16
    bool ok = true;
    RadixList rl;
    const bool smooth = radices(N, rl);
    if (smooth && N <= kGenTileL) {
        p->kind = kTileKind;
        p->rl = rl;
        ok = upload(&p->tw, twiddles(N));
        RadixList h;
        if (ok && N == 14400 && radices(N / 2, h) && h.n == 6 && h.R[0] == 3 && h.R[1] == 3 &&
            h.R[2] == 5 && h.R[3] == 5 && h.R[4] == 2 && h.R[5] == 16)
            ok = upload(&p->tw_half, twiddles(N / 2));
    } else if (smooth) {
        int d = (int)std::sqrt((double)N);
        while (d > 1 && (N % d || N / d > kGenTile)) --d;
        RadixList a, b;
        if (d > 1 && N % d == 0 && N / d <= kGenTile && radices(d, a) && radices(N / d, b)) {
            p->kind = kFourKind;
            p->N2 = d;
            p->N1 = N / d;
            p->rlA = a;
            p->rlB = b;
            ok = upload(&p->tw, twiddles(N)) && upload(&p->twA, twiddles(p->N2)) &&
                 upload(&p->twB, twiddles(p->N1));
        }
    }
    if (!p->kind) {
        // Bluestein with a power-of-two convolution length M >= 2N - 1 (fft.hip: M <= 2^20)
        long M = 1;
        while (M < 2L * N - 1) M <<= 1;
        if (M > (1L << 20)) {
            delete p;
            *status = SDRGPU_ERR_UNSUPPORTED;
            return nullptr;
        }
        p->kind = kBluKind;
        p->M = (int)M;
        std::vector<float2> w((size_t)N);
        std::vector<std::complex<double>> b((size_t)M, 0.0);
        for (long n = 0; n < N; ++n) {
            const long q = (long)((unsigned long long)n * (unsigned long long)n % (2ULL * N));
            const double ang = -M_PI * (double)q / (double)N;
            const std::complex<double> wn(std::cos(ang), std::sin(ang));
            w[(size_t)n] = make_float2((float)wn.real(), (float)wn.imag());
            b[(size_t)n] = std::conj(wn);
            if (n) b[(size_t)(M - n)] = std::conj(wn);
        }
        host_fft(b);
        std::vector<float2> bh((size_t)M);
        for (long m = 0; m < M; ++m)
            bh[(size_t)m] = make_float2((float)(b[(size_t)m].real() / M), (float)(b[(size_t)m].imag() / M));
        int st = SDRGPU_OK;
        p->inner = fft_plan_create((int)M, &st);
        ok = st == SDRGPU_OK && upload(&p->chirp, w) && upload(&p->bhat, bh);
    }
    if (!ok) {
        fftgen_plan_destroy(p);
        *status = SDRGPU_ERR_NOMEM;
        return nullptr;
    }
    *status = SDRGPU_OK;
    return p;
}

size_t fftgen_frame_scratch_bytes(void* plan) {
    auto* p = static_cast<GenFftPlan*>(plan);
    if (p->kind == kFourKind) return (size_t)p->N * sizeof(float2);
    if (p->kind == kBluKind)  // T and U, plus the inner plan's own slab if it has one
        return (size_t)p->M * sizeof(float2) * (fft_scratch_frames(p->inner) ? 3 : 2);
    return 0;
}

int fftgen_launch(void* plan, const FftFrames& fr, float2* out, int store_mode, float2* scratch,
                  size_t scratch_frames, hipStream_t s) {
    auto* p = static_cast<GenFftPlan*>(plan);
    if (fr.nframes <= 0) return SDRGPU_OK;
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
    const long N = p->N;
    auto advance = [&](FrameSrc& a, long f0) {
        if (frame_src_is_stream(a.mode)) a.first_end += f0 * a.hop;
        else if (a.mode == 0) a.in += f0 * N;
        else a.in_real += f0 * N;
    };
    if (p->kind == kTileKind) {
        GenTileArgs a{};
        a.src = src;
        a.nframes = fr.nframes;
        a.N = (int)N;
        const bool wave = N <= kGenTileW, large = N > kGenTile;
        a.B = large ? 1 : std::max(1, (wave ? kGenTileW : kGenTile) / (int)N);
        a.rl = p->rl;
        a.tw = p->tw;
        a.norm = p->norm;
        a.store_mode = store_mode;
        a.out = out;
        const long blocks = (fr.nframes + a.B - 1) / a.B;
        if (p->tw_half && (store_mode == 1 || store_mode == 4) && src.mode == 2 &&
            ((uintptr_t)src.in_real & 7) == 0) {
            // examples/fft.rs's rfft: real frames as 7,200 complex points, packed transform
            static const bool attr = hipFuncSetAttribute(
                (const void*)gen_rfft_half_kernel<kRfftBlk, kRfftTile, 7200, 3, 3, 5, 5, 2, 16>,
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lp_bytes<kRfftTile>(kRfftTile)) == hipSuccess;
            if (!attr) return SDRGPU_ERR_LAUNCH;
            GenTileArgs h = a;
            h.src.mode = 0;
            h.src.in = reinterpret_cast<const float2*>(src.in_real);
            constexpr int B2 = kRfftTile / 7200;
            hipLaunchKernelGGL((gen_rfft_half_kernel<kRfftBlk, kRfftTile, 7200, 3, 3, 5, 5, 2, 16>),
                               dim3((unsigned)((fr.nframes + B2 - 1) / B2)), dim3(kRfftBlk),
                               lp_bytes<kRfftTile>(B2 * 7200), s, h, (const float2*)p->tw_half);
        } else if (large && N == 14400 && p->rl.n == 6 && p->rl.R[0] == 3 && p->rl.R[1] == 3 &&
            p->rl.R[2] == 5 && p->rl.R[3] == 5 && p->rl.R[4] == 4 && p->rl.R[5] == 16) {
            // examples/fft.rs: take(0.1) at 144 kHz, compile-time plan
            static const bool attr = hipFuncSetAttribute(
                (const void*)gen_fixed_kernel<kGenBlockL, kGenTileL, 14400, 3, 3, 5, 5, 4, 16>,
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lp_bytes<kGenTileL>(kGenTileL)) == hipSuccess;
            if (!attr) return SDRGPU_ERR_LAUNCH;
            hipLaunchKernelGGL((gen_fixed_kernel<kGenBlockL, kGenTileL, 14400, 3, 3, 5, 5, 4, 16>),
                               dim3((unsigned)blocks), dim3(kGenBlockL), lp_bytes<kGenTileL>(N), s, a);
        } else if (large) {
            static const bool attr = hipFuncSetAttribute(
                (const void*)gen_tile_kernel<kGenBlockL, kGenTileL>,
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lp_bytes<kGenTileL>(kGenTileL)) == hipSuccess;
            if (!attr) return SDRGPU_ERR_LAUNCH;
            hipLaunchKernelGGL((gen_tile_kernel<kGenBlockL, kGenTileL>), dim3((unsigned)blocks),
                               dim3(kGenBlockL), lp_bytes<kGenTileL>(N), s, a);
        } else if (N == 1000 && a.B == 1 && p->rl.n == 4 && p->rl.R[0] == 5 && p->rl.R[1] == 5 &&
                   p->rl.R[2] == 5 && p->rl.R[3] == 8)  // examples/live.rs: compile-time plan
            hipLaunchKernelGGL((gen_fixed_kernel<kLiveBlk, kLiveTile, 1000, 5, 5, 5, 8>),
                               dim3((unsigned)((fr.nframes + kLiveTile / 1000 - 1) / (kLiveTile / 1000))),
                               dim3(kLiveBlk), lp_bytes<kLiveTile>(kLiveTile / 1000 * 1000), s, a);
        else if (wave)
            hipLaunchKernelGGL((gen_tile_kernel<64, kGenTileW>), dim3((unsigned)blocks), dim3(64),
                               lp_bytes<kGenTileW>(a.B * N), s, a);
        else
            hipLaunchKernelGGL((gen_tile_kernel<kGenBlock, kGenTile>), dim3((unsigned)blocks),
                               dim3(kGenBlock), lp_bytes<kGenTile>(a.B * N), s, a);
        SDRGPU_LAUNCH_CHECK();
        return SDRGPU_OK;
    }
    if (!scratch || scratch_frames == 0) return SDRGPU_ERR_UNSUPPORTED;
    if (p->kind == kFourKind) {
        Gen4Args a{};
        a.N = (int)N;
        a.N1 = p->N1;
        a.N2 = p->N2;
        a.rlA = p->rlA;
        a.rlB = p->rlB;
        a.twA = p->twA;
        a.twB = p->twB;
        a.twN = p->tw;
        a.norm = p->norm;
        a.store_mode = store_mode;
        a.scratch = scratch;
        const int CA = kGenTile / p->N2, CB = kGenTile / p->N1;
        const long ta = (p->N1 + CA - 1) / CA, tb = (p->N2 + CB - 1) / CB;
        for (long f0 = 0; f0 < fr.nframes; f0 += (long)scratch_frames) {
            const long nf = std::min((long)scratch_frames, fr.nframes - f0);
            a.src = src;
            advance(a.src, f0);
            a.nframes = nf;
            a.out = store_advance(out, f0, N, store_mode);
            hipLaunchKernelGGL(gen4_pass_a, dim3((unsigned)(nf * ta)), dim3(kGenBlock),
                               lp_bytes<kGenTile>(std::min(CA, p->N1) * p->N2), s, a);
            SDRGPU_LAUNCH_CHECK();
            hipLaunchKernelGGL(gen4_pass_b, dim3((unsigned)(nf * tb)), dim3(kGenBlock),
                               lp_bytes<kGenTile>(std::min(CB, p->N2) * p->N1), s, a);
            SDRGPU_LAUNCH_CHECK();
        }
        return SDRGPU_OK;
    }
    // Bluestein: per batch T and U (nf x M each), then (if the inner plan needs one) its slab;
    // every transform runs T -> U (the power-of-two kernels are not in place)
    const long M = p->M;
    const bool inner_scratch = fft_scratch_frames(p->inner) != 0;
    float2* U = scratch + (long)scratch_frames * M;
    float2* inner_buf = inner_scratch ? scratch + 2L * (long)scratch_frames * M : nullptr;
    BluArgs a{};
    a.N = (int)N;
    a.M = (int)M;
    a.chirp = p->chirp;
    a.bhat = p->bhat;
    a.T = scratch;
    a.U = U;
    a.norm = p->norm;
    a.store_mode = store_mode;
    for (long f0 = 0; f0 < fr.nframes; f0 += (long)scratch_frames) {
        const long nf = std::min((long)scratch_frames, fr.nframes - f0);
        a.src = src;
        advance(a.src, f0);
        a.nframes = nf;
        a.out = store_advance(out, f0, N, store_mode);
        const unsigned g = (unsigned)std::min<long>(4096, (nf * M + 255) / 256);
        hipLaunchKernelGGL(blu_pre, dim3(g), dim3(256), 0, s, a);
        SDRGPU_LAUNCH_CHECK();
        FftFrames in{};
        in.mode = 0;
        in.in = scratch;
        in.nframes = nf;
        int st = fft_launch(p->inner, in, U, 2, inner_buf, inner_scratch ? scratch_frames : 0, s);
        if (st) return st;
        hipLaunchKernelGGL(blu_mid, dim3(g), dim3(256), 0, s, a);
        SDRGPU_LAUNCH_CHECK();
        if ((st = fft_launch(p->inner, in, U, 2, inner_buf, inner_scratch ? scratch_frames : 0, s)))
            return st;
        const unsigned gp = (unsigned)std::min<long>(4096, (nf * N + 255) / 256);
        hipLaunchKernelGGL(blu_post, dim3(gp), dim3(256), 0, s, a);
        SDRGPU_LAUNCH_CHECK();
    }
    return SDRGPU_OK;
}

}  // namespace sdrgpu
