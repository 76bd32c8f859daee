// fir_os.hip -- polyphase overlap-save FIR / FIR-decimate for gfx950.
//
// Same semantics as fir_direct.hip (Fir::apply + Decimate, reference
// src/filter/fir.rs:23-32 and src/signal/adapters/mod.rs:30-37) for complex samples.
//
// Why: direct form costs 4*K flops per kept output (1020 flop / output at K=255), which
// puts configs[1] on the FP32 roof, not the HBM roof.  Here each kept
// output costs ~75 flop (a few FFT butterflies), so the kernel can stream at HBM speed.
//
// Math.  With decimation D, y[m] = sum_b sum_i h_b[i] s_b[m-i], h_b[i] = h[b+iD],
// s_b[m'] = x[i0 + m'D - b] (D polyphase branches, each a T = ceil(K/D)-tap FIR at the
// output rate).  A workgroup owns M consecutive kept outputs and reads ONE contiguous
// 4096-sample input window: the D branch windows of L = 4096/D samples each.  It runs D
// forward L-point FFTs, multiplies by the branch spectra H_b (1/L folded in) and sums
// them -- the decimation happens in the frequency domain for free -- then one inverse
// L-point FFT yields L circular outputs of which the last M = L - (>= T-1) are the linear
// convolution.  For K=255, D=4: L = 1024, M = 960 kept outputs per 4096 (3840 new) inputs.
//
// Layout / schedule (256 lanes, 16 complex values per lane, LDS = D x L (+pad) c64):
//   P1 radix-16 from HBM: lane t reads x[base + t + 256 r] (r<16) -- 64 consecutive
//      samples per wave-instruction -- so lane t is (branch D-1-t%D, index t/D);
//   P2 radix-16 LDS->LDS; P3 radix-L/256: lane j owns bins j + 256 r of ALL branches, so
//      the branch sum Z = sum_b X_b H_b happens in registers;
//   I1 inverse radix-L/256 straight from those registers; I2, I3 radix-16; I3 stores the
//      kept outputs coalesced.  Stockham autosort order, twiddles from one 4096-entry
//      table + recurrence.  LDS index padded (i + i/16, branch stride L + L/16 + 4) so
//      every pass is (nearly) bank-conflict free.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fft_device.hpp"
#include "fir_kernels.hpp"

namespace sdrgpu {

using namespace fftd;

namespace {

constexpr int kOsBlock = 256;
constexpr int kOsPoints = 4096;  // D * L

__device__ __forceinline__ int opad(int i) { return i + (i >> 4); }

struct OsParams {
    const float2* in;
    long ld_in, n_in;
    const float2* hist;
    float2* hist_next;
    long i0, n_out;
    int K;
    int M;                       // kept outputs per workgroup
    const float2* H;             // D x L branch spectra (1/L folded in)
    const float2* tw;            // exp(-2 pi i m / 4096), m < 4096
    float2* out;
    long ld_out;
};

template <int D>
__global__ __launch_bounds__(kOsBlock) void fir_os_kernel(OsParams p) {
    constexpr int L = kOsPoints / D;
    constexpr int R3 = L / 256;              // radix of the last forward / first inverse pass
    constexpr int LP = L + L / 16 + 4;       // padded branch stride (elements)
    __shared__ float2 lds[D * LP];

    const int t = threadIdx.x;
    const long ch = blockIdx.y;
    const float2* __restrict__ in = p.in + ch * p.ld_in;
    const float2* __restrict__ hist = p.hist + ch * (long)(p.K - 1);
    float2* __restrict__ out = p.out + ch * p.ld_out;
    const float2* __restrict__ tw = p.tw;
    const int K = p.K;

    const long m0 = (long)blockIdx.x * p.M;   // first kept output of this workgroup
    if (m0 < p.n_out) {
        // input window: x[base + t + 256 r]; base = i0 + (m0 + M - L) * D - (D - 1)
        const long base = p.i0 + (m0 + p.M - L) * (long)D - (D - 1);
        float2 v[16];

        // ---- P1: radix-16, Ns = 1, from HBM ----
        {
            const long g0 = base + t;
            if (g0 >= 0 && g0 + 256 * 15 < p.n_in) {
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = in[g0 + 256 * r];
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const long g = g0 + 256 * r;
                    float2 x = make_float2(0.f, 0.f);
                    if (g >= 0) {
                        if (g < p.n_in) x = in[g];
                    } else if (g >= -(long)(K - 1)) {
                        x = hist[g + (K - 1)];
                    }
                    v[r] = x;
                }
            }
            Dft<16, false>::run(v);
            const int b = D - 1 - (t % D), j = t / D;
            float2* dst = lds + b * LP;
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[opad(16 * j + r)] = v[r];
        }
        __syncthreads();

        // ---- P2: radix-16, Ns = 16, LDS in place ----
        {
            constexpr int NB = L / 16;  // butterflies per branch
            const int b = t / NB, j = t % NB;
            float2* buf = lds + b * LP;
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = buf[opad(j + NB * r)];
            const int k = j & 15;
            twiddle<16, false>(v, tw, k * (kOsPoints / 256));
            Dft<16, false>::run(v);
            __syncthreads();
            const int o = (j >> 4) * 256 + k;
#pragma unroll
            for (int r = 0; r < 16; ++r) buf[opad(o + 16 * r)] = v[r];
        }
        __syncthreads();

        // ---- P3: radix-R3, Ns = 256; lane j owns bins j + 256 r of every branch ----
        float2 z[R3];
        {
            const int j = t;
#pragma unroll
            for (int r = 0; r < R3; ++r) z[r] = make_float2(0.f, 0.f);
#pragma unroll
            for (int b = 0; b < D; ++b) {
                float2 w[R3];
                const float2* buf = lds + b * LP;
#pragma unroll
                for (int r = 0; r < R3; ++r) w[r] = buf[opad(j + 256 * r)];
                twiddle<R3, false>(w, tw, j * D);
                Dft<R3, false>::run(w);
                const float2* Hb = p.H + b * L;
#pragma unroll
                for (int r = 0; r < R3; ++r) {
                    const float2 h = Hb[j + 256 * r];
                    z[r].x = fmaf(w[r].x, h.x, fmaf(-w[r].y, h.y, z[r].x));
                    z[r].y = fmaf(w[r].x, h.y, fmaf(w[r].y, h.x, z[r].y));
                }
            }
        }
        __syncthreads();  // all P3 reads done before I1 overwrites branch 0

        // ---- I1: inverse radix-R3, Ns = 1, from registers ----
        {
            const int j = t;
            Dft<R3, true>::run(z);
#pragma unroll
            for (int r = 0; r < R3; ++r) lds[opad(j * R3 + r)] = z[r];
        }
        __syncthreads();

        // ---- I2: inverse radix-16, Ns = R3 ----
        constexpr int NBI = L / 16;
        if (t < NBI) {
            const int j = t;
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = lds[opad(j + NBI * r)];
            const int k = j % R3;
            twiddle<16, true>(v, tw, k * (kOsPoints / (R3 * 16)));
            Dft<16, true>::run(v);
        }
        __syncthreads();
        if (t < NBI) {
            const int j = t;
            const int k = j % R3;
            const int o = (j / R3) * R3 * 16 + k;
#pragma unroll
            for (int r = 0; r < 16; ++r) lds[opad(o + R3 * r)] = v[r];
        }
        __syncthreads();

        // ---- I3: inverse radix-16, Ns = L/16; outputs i = j + (L/16) r ----
        if (t < NBI) {
            const int j = t;
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = lds[opad(j + NBI * r)];
            twiddle<16, true>(v, tw, j * D);
            Dft<16, true>::run(v);
            const int skip = L - p.M;  // circular-wrap outputs
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = j + NBI * r;
                const long m = m0 + (i - skip);
                if (i >= skip && m < p.n_out) out[m] = v[r];
            }
        }
    }

    if (blockIdx.x == gridDim.x - 1) {  // stream history carry (see fir_direct.hip)
        float2* hn = p.hist_next + ch * (long)(K - 1);
        for (int jj = t; jj < K - 1; jj += kOsBlock) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

// ---------------------------------------------------------------------------------
// v2 (D in {4, 8}, L = 4096/D <= 1024): persistent workgroups with software pipelining.
// Each workgroup walks blocks q = blockIdx.x, +gridDim.x, ...; it issues the NEXT block's
// 16 loads per lane as soon as the forward passes are done, so they fly under
// I1..I5 of the current block (issued after P3, which is the last pass that loads
// the branch spectra H from global: the hardware's in-order vmcnt would otherwise make
// those loads wait for the prefetch).  Each pass's twiddle base is loaded once into
// registers before the loop, so the inverse passes issue no VMEM load at all.  The inverse L-point FFT is radix-R3 from registers, then four radix-4
// Stockham passes ping-ponging between two LDS regions with all 256 lanes busy.
template <int D>
__device__ __forceinline__ void os2_load(float2 (&v)[16], const float2* __restrict__ in,
                                         const float2* __restrict__ hist, long n_in, int K,
                                         long g0) {
    if (g0 >= 0 && g0 + 256 * 15 < n_in) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = in[g0 + 256 * r];
    } else {
        // edge blocks (stream start with history, ragged tail): branch-free selects
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const long g = g0 + 256 * r;
            const bool inb = (g >= 0) & (g < n_in);
            const bool inh = (g < 0) & (g >= -(long)(K - 1));
            const float2 x = in[inb ? g : 0];
            const float2 xh = hist[inh ? g + (K - 1) : 0];
            v[r] = inb ? x : (inh ? xh : make_float2(0.f, 0.f));
        }
    }
}

// HR: the lane's D*R3 branch-spectrum values H_b[t + 256 r] are loaded once into registers
// instead of from L2 every window (the per-window H loads double the vector-memory
// instructions of the stream)
template <int D, bool PF, int W, bool HR = false>
__global__ __launch_bounds__(kOsBlock, W) void fir_os2_kernel(OsParams p, long nblk) {
    constexpr int L = kOsPoints / D;
    constexpr int R3 = L / 256;
    constexpr int LP = L + L / 16 + 4;
    constexpr int NB = L / 16;   // forward radix-16 butterflies per branch
    constexpr int NI = L / 4;    // inverse radix-4 butterflies (<= 256)
    constexpr int IB = L + L / 16 + 8;  // offset of the second inverse buffer
    static_assert(D * 16 * NB == 4096 && NI <= kOsBlock && 2 * IB <= D * LP, "geometry");
    static_assert(NB % 16 == 0 && NI % 16 == 0, "padded strides need multiples of 16");
    // padded offset of a multiple of 16: opad(i + n) = opad(i) + ps(n)
    constexpr auto ps = [](int n) { return n + n / 16; };
    __shared__ float2 lds[D * LP];
    float2* const bufA = lds;
    float2* const bufB = lds + IB;

    const long ch = blockIdx.y;
    const float2* __restrict__ in = p.in + ch * p.ld_in;
    const float2* __restrict__ hist = p.hist + ch * (long)(p.K - 1);
    float2* __restrict__ out = p.out + ch * p.ld_out;
    const float2* __restrict__ tw = p.tw;
    const int K = p.K;
    const int skip = L - p.M;

    // ---- per-lane twiddle bases (loaded once; the loop body loads only H and samples) ----
    const int t0 = threadIdx.x;
    const float2 w2b = tw[16 * ((t0 % NB) & 15)];
    const float2 w3b = tw[t0 * D];
    float2 wib[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int Ns = R3 << (2 * s);
        const int k = (t0 % NI) % Ns;
        wib[s] = conjf2(tw[k * (kOsPoints / (4 * Ns))]);
    }

    float2 hreg[HR ? D * R3 : 1];
    if (HR) {
#pragma unroll
        for (int b = 0; b < D; ++b)
#pragma unroll
            for (int r = 0; r < R3; ++r) hreg[HR ? b * R3 + r : 0] = p.H[b * L + 256 * r + t0];
    }
    float2 v[16];
    long q = blockIdx.x;
    const long hop = (long)p.M * D;
    long base = p.i0 + (q * p.M + p.M - L) * (long)D - (D - 1);
    if (PF && q < nblk) os2_load<D>(v, in, hist, p.n_in, K, base + t0);

#pragma unroll 1
    for (; q < nblk; q += gridDim.x, base += hop * gridDim.x) {
        // opaque per-iteration copy of the lane id: keeps the ~20 per-lane LDS/H address
        // computations inside the loop instead of hoisting them into live registers
        int t = t0;
        asm volatile("" : "+v"(t));
        // same for the twiddle bases: their powers are recomputed per block (cheap VALU)
        // rather than hoisted into ~60 loop-invariant registers
        float2 w2 = w2b, w3 = w3b, wi[4] = {wib[0], wib[1], wib[2], wib[3]};
        asm volatile("" : "+v"(w2.x), "+v"(w2.y), "+v"(w3.x), "+v"(w3.y));
        asm volatile("" : "+v"(wi[0].x), "+v"(wi[0].y), "+v"(wi[1].x), "+v"(wi[1].y),
                          "+v"(wi[2].x), "+v"(wi[2].y), "+v"(wi[3].x), "+v"(wi[3].y));

        // ---- P1: radix-16 on the (prefetched) samples ----
        if (!PF) os2_load<D>(v, in, hist, p.n_in, K, base + t);
        Dft<16, false>::run(v);
        {
            const int b = D - 1 - (t % D), j = t / D;
            float2* dst = lds + b * LP + 17 * j;           // opad(16 j + r) = 17 j + r
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = v[r];
        }
        __syncthreads();

        float2 u[16];
        // ---- P2: radix-16, Ns = 16 ----
        {
            const int b = t / NB, j = t % NB;
            float2* rd = lds + b * LP + opad(j);
#pragma unroll
            for (int r = 0; r < 16; ++r) u[r] = rd[ps(NB) * r];
            twiddle_tree<16>(u, w2);
            Dft<16, false>::run(u);
            __syncthreads();
            float2* wt = lds + b * LP + opad((j >> 4) * 256 + (j & 15));
#pragma unroll
            for (int r = 0; r < 16; ++r) wt[17 * r] = u[r];
        }
        __syncthreads();

        // ---- P3: radix-R3 per branch, multiply by H_b, sum over branches ----
        float2 z[R3];
#pragma unroll
        for (int r = 0; r < R3; ++r) z[r] = make_float2(0.f, 0.f);
        {
            const float2* rd0 = lds + opad(t);
            const float2* H = p.H + t;
#pragma unroll
            for (int b = 0; b < D; ++b) {
                float2 w[R3];
#pragma unroll
                for (int r = 0; r < R3; ++r) w[r] = rd0[b * LP + 272 * r];
                if (R3 > 1) twiddle_tree<R3>(w, w3);
                Dft<R3, false>::run(w);
#pragma unroll
                for (int r = 0; r < R3; ++r) {
                    const float2 h = HR ? hreg[HR ? b * R3 + r : 0] : H[b * L + 256 * r];
                    z[r].x = fmaf(w[r].x, h.x, fmaf(-w[r].y, h.y, z[r].x));
                    z[r].y = fmaf(w[r].x, h.y, fmaf(w[r].y, h.x, z[r].y));
                }
            }
        }
        // ---- prefetch the next block: flies under I1..I5 (no VMEM loads there) ----
        if (PF && q + gridDim.x < nblk) os2_load<D>(v, in, hist, p.n_in, K, base + hop * gridDim.x + t);
        __syncthreads();

        // ---- I1: inverse radix-R3, Ns = 1 ----
        Dft<R3, true>::run(z);
        {
            float2* wt = bufA + opad(t * R3);
#pragma unroll
            for (int r = 0; r < R3; ++r) wt[r] = z[r];
        }
        __syncthreads();

        // ---- I2..I4: inverse radix-4, Ns = R3, 4R3, 16R3 (ping-pong A/B) ----
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            const int Ns = R3 << (2 * s);
            const float2* src = (s & 1) ? bufB : bufA;
            float2* dst = (s & 1) ? bufA : bufB;
            if (t < NI) {
                const int j = t, k = j % Ns;
                const float2* rd = src + opad(j);
                float2 a0 = rd[0], a1 = rd[ps(NI)], a2 = rd[2 * ps(NI)], a3 = rd[3 * ps(NI)];
                const float2 w = wi[s], w2_ = cmul(w, w), w3_ = cmul(w2_, w);
                a1 = cmul(a1, w);
                a2 = cmul(a2, w2_);
                a3 = cmul(a3, w3_);
                dft4<true>(a0, a1, a2, a3);
                const int o = (j / Ns) * 4 * Ns + k;
                dst[opad(o)] = a0;
                dst[opad(o + Ns)] = a1;
                dst[opad(o + 2 * Ns)] = a2;
                dst[opad(o + 3 * Ns)] = a3;
            }
            __syncthreads();
        }

        // ---- I5: inverse radix-4, Ns = L/4; outputs i = j + (L/4) r, stored coalesced ----
        if (t < NI) {
            const int j = t;
            const float2* rd = bufB + opad(j);
            float2 a0 = rd[0], a1 = rd[ps(NI)], a2 = rd[2 * ps(NI)], a3 = rd[3 * ps(NI)];
            const float2 w = wi[3], w2_ = cmul(w, w), w3_ = cmul(w2_, w);
            a1 = cmul(a1, w);
            a2 = cmul(a2, w2_);
            a3 = cmul(a3, w3_);
            dft4<true>(a0, a1, a2, a3);
            const long m0 = q * p.M - skip + j;
            float2* o = out + m0;
            if (j >= skip && m0 < p.n_out) o[0] = a0;
            if (j + NI >= skip && m0 + NI < p.n_out) o[NI] = a1;
            if (j + 2 * NI >= skip && m0 + 2 * NI < p.n_out) o[2 * NI] = a2;
            if (j + 3 * NI >= skip && m0 + 3 * NI < p.n_out) o[3 * NI] = a3;
        }
        __syncthreads();  // I5 reads of bufB finish before the next P1 writes
    }

    if (blockIdx.x == gridDim.x - 1) {  // stream history carry (see fir_direct.hip)
        float2* hn = p.hist_next + ch * (long)(K - 1);
        for (int jj = t0; jj < K - 1; jj += kOsBlock) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

// ---------------------------------------------------------------------------------
// v3: like v2 but each persistent iteration processes NB consecutive blocks interleaved
// through every pass (NB x the independent work between barriers, 1/NB the barriers per
// block; LDS = NB x D x L).  Loads are issued at the top of the iteration for all NB blocks.
// ABL (debug ablation): 0 = full kernel, 1 = memory only (loads -> stores, no FFT work),
// 2 = compute only (no HBM loads: samples synthesised from the lane id)
template <int D, int NB, int W, int ABL = 0>
__global__ __launch_bounds__(kOsBlock, W) void fir_os3_kernel(OsParams p, long nblk) {
    constexpr int L = kOsPoints / D;
    constexpr int R3 = L / 256;
    constexpr int LP = L + L / 16 + 4;
    constexpr int BR = L / 16;   // forward radix-16 butterflies per branch
    constexpr int NI = L / 4;    // inverse radix-4 butterflies (<= 256)
    constexpr int IB = L + L / 16 + 8;
    constexpr int SB = D * LP;   // LDS elements per block
    static_assert(D * 16 * BR == 4096 && NI <= kOsBlock && 2 * IB <= SB, "geometry");
    static_assert(BR % 16 == 0 && NI % 16 == 0, "padded strides need multiples of 16");
    constexpr auto ps = [](int n) { return n + n / 16; };
    __shared__ float2 lds[NB * SB];

    const long ch = blockIdx.y;
    const float2* __restrict__ in = p.in + ch * p.ld_in;
    const float2* __restrict__ hist = p.hist + ch * (long)(p.K - 1);
    float2* __restrict__ out = p.out + ch * p.ld_out;
    const float2* __restrict__ tw = p.tw;
    const int K = p.K;
    const int skip = L - p.M;

    const int t0 = threadIdx.x;
    const float2 w2b = tw[16 * ((t0 % BR) & 15)];
    const float2 w3b = tw[t0 * D];
    float2 wib[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int Ns = R3 << (2 * s);
        const int k = (t0 % NI) % Ns;
        wib[s] = conjf2(tw[k * (kOsPoints / (4 * Ns))]);
    }
    const long nsb = (nblk + NB - 1) / NB;
    const long hop = (long)p.M * D;

#pragma unroll 1
    for (long sb = blockIdx.x; sb < nsb; sb += gridDim.x) {
        int t = t0;
        asm volatile("" : "+v"(t));
        float2 w2 = w2b, w3 = w3b, wi[4] = {wib[0], wib[1], wib[2], wib[3]};
        asm volatile("" : "+v"(w2.x), "+v"(w2.y), "+v"(w3.x), "+v"(w3.y));
        asm volatile("" : "+v"(wi[0].x), "+v"(wi[0].y), "+v"(wi[1].x), "+v"(wi[1].y),
                          "+v"(wi[2].x), "+v"(wi[2].y), "+v"(wi[3].x), "+v"(wi[3].y));
        const long q0 = sb * NB;
        const long base0 = p.i0 + (q0 * p.M + p.M - L) * (long)D - (D - 1);

        // ---- loads for all NB blocks, then P1 radix-16 ----
        float2 v[NB][16];
        if (ABL == 2) {
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
                for (int r = 0; r < 16; ++r) v[nb][r] = make_float2((float)(t + r), (float)(sb + nb));
        } else {
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) os2_load<D>(v[nb], in, hist, p.n_in, K, base0 + nb * hop + t);
        }
        if (ABL == 1) {
            // memory-only: store the loaded samples where I5 would store outputs
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const long m0 = (q0 + nb) * p.M - skip + t;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = t + NI * r;
                    if (i >= skip && m0 + NI * r < p.n_out && t < NI)
                        out[m0 + NI * r] = cadd(v[nb][r], cadd(v[nb][r + 4], cadd(v[nb][r + 8], v[nb][r + 12])));
                }
            }
            continue;
        }
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            Dft<16, false>::run(v[nb]);
            const int b = D - 1 - (t % D), j = t / D;
            float2* dst = lds + nb * SB + b * LP + 17 * j;
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[r] = v[nb][r];
        }
        __syncthreads();

        // ---- P2: radix-16, Ns = 16 (in place) ----
        {
            const int b = t / BR, j = t % BR;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const float2* rd = lds + nb * SB + b * LP + opad(j);
#pragma unroll
                for (int r = 0; r < 16; ++r) v[nb][r] = rd[ps(BR) * r];
                twiddle_tree<16>(v[nb], w2);
                Dft<16, false>::run(v[nb]);
            }
            __syncthreads();
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                float2* wt = lds + nb * SB + b * LP + opad((j >> 4) * 256 + (j & 15));
#pragma unroll
                for (int r = 0; r < 16; ++r) wt[17 * r] = v[nb][r];
            }
        }
        __syncthreads();

        // ---- P3 + branch sum ----
        float2 z[NB][R3];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
            for (int r = 0; r < R3; ++r) z[nb][r] = make_float2(0.f, 0.f);
            const float2* rd0 = lds + nb * SB + opad(t);
            const float2* H = p.H + t;
#pragma unroll
            for (int b = 0; b < D; ++b) {
                float2 w[R3];
#pragma unroll
                for (int r = 0; r < R3; ++r) w[r] = rd0[b * LP + 272 * r];
                if (R3 > 1) twiddle_tree<R3>(w, w3);
                Dft<R3, false>::run(w);
#pragma unroll
                for (int r = 0; r < R3; ++r) {
                    const float2 h = H[b * L + 256 * r];
                    z[nb][r].x = fmaf(w[r].x, h.x, fmaf(-w[r].y, h.y, z[nb][r].x));
                    z[nb][r].y = fmaf(w[r].x, h.y, fmaf(w[r].y, h.x, z[nb][r].y));
                }
            }
        }
        __syncthreads();

        // ---- I1 ----
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            Dft<R3, true>::run(z[nb]);
            float2* wt = lds + nb * SB + opad(t * R3);
#pragma unroll
            for (int r = 0; r < R3; ++r) wt[r] = z[nb][r];
        }
        __syncthreads();

        // ---- I2..I4 (ping-pong A/B inside each block's LDS) ----
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            const int Ns = R3 << (2 * s);
            if (t < NI) {
                const int j = t, k = j % Ns;
                const float2 w = wi[s], w2_ = cmul(w, w), w3_ = cmul(w2_, w);
                const int o = (j / Ns) * 4 * Ns + k;
#pragma unroll
                for (int nb = 0; nb < NB; ++nb) {
                    const float2* src = lds + nb * SB + ((s & 1) ? IB : 0);
                    float2* dst = lds + nb * SB + ((s & 1) ? 0 : IB);
                    const float2* rd = src + opad(j);
                    float2 a0 = rd[0], a1 = rd[ps(NI)], a2 = rd[2 * ps(NI)], a3 = rd[3 * ps(NI)];
                    a1 = cmul(a1, w);
                    a2 = cmul(a2, w2_);
                    a3 = cmul(a3, w3_);
                    dft4<true>(a0, a1, a2, a3);
                    dst[opad(o)] = a0;
                    dst[opad(o + Ns)] = a1;
                    dst[opad(o + 2 * Ns)] = a2;
                    dst[opad(o + 3 * Ns)] = a3;
                }
            }
            __syncthreads();
        }

        // ---- I5 -> global ----
        if (t < NI) {
            const int j = t;
            const float2 w = wi[3], w2_ = cmul(w, w), w3_ = cmul(w2_, w);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const float2* rd = lds + nb * SB + IB + opad(j);
                float2 a0 = rd[0], a1 = rd[ps(NI)], a2 = rd[2 * ps(NI)], a3 = rd[3 * ps(NI)];
                a1 = cmul(a1, w);
                a2 = cmul(a2, w2_);
                a3 = cmul(a3, w3_);
                dft4<true>(a0, a1, a2, a3);
                const long m0 = (q0 + nb) * p.M - skip + j;
                float2* o = out + m0;
                if (j >= skip && m0 < p.n_out) o[0] = a0;
                if (j + NI >= skip && m0 + NI < p.n_out) o[NI] = a1;
                if (j + 2 * NI >= skip && m0 + 2 * NI < p.n_out) o[2 * NI] = a2;
                if (j + 3 * NI >= skip && m0 + 3 * NI < p.n_out) o[3 * NI] = a3;
            }
        }
        __syncthreads();
    }

    if (blockIdx.x == gridDim.x - 1) {
        float2* hn = p.hist_next + ch * (long)(K - 1);
        for (int jj = t0; jj < K - 1; jj += kOsBlock) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

// ---------------------------------------------------------------------------------
// v4 (D = 4, L = 1024): 512-lane workgroups, 8 points per lane, radix-8 passes, so that
// 4 workgroups (8 waves/SIMD, <= 64 VGPRs) share a CU and hide LDS/barrier latency.
//   forward per branch 8*8*8*2: P1 radix-8 from HBM (lane t: branch 3-t%4, x[base+t+512r]),
//   P2 radix-8 (Ns 8), P3 radix-8 (Ns 64), P4 radix-2 (Ns 512) with lane j owning bins j and
//   j+512 of all 4 branches -> Z = sum_b X_b H_b in registers;
//   inverse 2*8*8*8: I1 radix-2 from registers, I2/I3/I4 radix-8 on 128 lanes, I4 -> HBM.
constexpr int kOs4Block = 512;

template <int W>
__global__ __launch_bounds__(kOs4Block, W) void fir_os4_kernel(OsParams p, long nblk) {
    constexpr int D = 4, L = 1024, LP = L + L / 16 + 4;
    __shared__ float2 lds[D * LP];
    float2* const bufA = lds;
    float2* const bufB = lds + (L + L / 16 + 8);

    const long ch = blockIdx.y;
    const float2* __restrict__ in = p.in + ch * p.ld_in;
    const float2* __restrict__ hist = p.hist + ch * (long)(p.K - 1);
    float2* __restrict__ out = p.out + ch * p.ld_out;
    const float2* __restrict__ tw = p.tw;
    const int K = p.K;
    const int skip = L - p.M;
    const int t0 = threadIdx.x;

#pragma unroll 1
    for (long q = blockIdx.x; q < nblk; q += gridDim.x) {
        int t = t0;
        asm volatile("" : "+v"(t));
        // per-lane twiddle bases, re-read each block (L1 hits; no prefetch to protect here):
        // P2 W^(64 (j&7)), P3 W^(8 (j&63)), P4 W^(4 t), I2 conj W^(256 (j&1)),
        // I3 conj W^(32 (j&15)), I4 conj W^(4 j)   (W = W4096, j = t & 127)
        const int jb = t & 127;
        const long base = p.i0 + (q * p.M + p.M - L) * (long)D - (D - 1);
        float2 v[8];

        // ---- P1: radix-8 from HBM ----
        {
            const long g0 = base + t;
            if (g0 >= 0 && g0 + 512 * 7 < p.n_in) {
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = in[g0 + 512 * r];
            } else {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const long g = g0 + 512 * r;
                    const bool inb = (g >= 0) & (g < p.n_in);
                    const bool inh = (g < 0) & (g >= -(long)(K - 1));
                    const float2 x = in[inb ? g : 0];
                    const float2 xh = hist[inh ? g + (K - 1) : 0];
                    v[r] = inb ? x : (inh ? xh : make_float2(0.f, 0.f));
                }
            }
            Dft<8, false>::run(v);
            const int b = 3 - (t & 3), j = t >> 2;
            float2* dst = lds + b * LP;
#pragma unroll
            for (int r = 0; r < 8; ++r) dst[opad(8 * j + r)] = v[r];
        }
        __syncthreads();
        // ---- P2: radix-8, Ns = 8 (in place) ----
        {
            const int b = t >> 7, j = t & 127, k = j & 7;
            float2* buf = lds + b * LP;
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = buf[opad(j + 128 * r)];
            twiddle_tree<8>(v, tw[64 * (jb & 7)]);
            Dft<8, false>::run(v);
            __syncthreads();
            const int o = (j >> 3) * 64 + k;
#pragma unroll
            for (int r = 0; r < 8; ++r) buf[opad(o + 8 * r)] = v[r];
        }
        __syncthreads();
        // ---- P3: radix-8, Ns = 64 (in place) ----
        {
            const int b = t >> 7, j = t & 127, k = j & 63;
            float2* buf = lds + b * LP;
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = buf[opad(j + 128 * r)];
            twiddle_tree<8>(v, tw[8 * (jb & 63)]);
            Dft<8, false>::run(v);
            __syncthreads();
            const int o = (j >> 6) * 512 + k;
#pragma unroll
            for (int r = 0; r < 8; ++r) buf[opad(o + 64 * r)] = v[r];
        }
        __syncthreads();
        // ---- P4: radix-2, Ns = 512: lane j owns bins j, j+512 of all branches ----
        float2 z0 = make_float2(0.f, 0.f), z1 = make_float2(0.f, 0.f);
        {
            const int j = t;
            const float2* H = p.H + j;
            const float2 w4 = tw[4 * j];
#pragma unroll
            for (int b = 0; b < D; ++b) {
                const float2* buf = lds + b * LP;
                float2 a0 = buf[opad(j)], a1 = cmul(buf[opad(j + 512)], w4);
                dft2<false>(a0, a1);
                const float2 h0 = H[b * L], h1 = H[b * L + 512];
                z0.x = fmaf(a0.x, h0.x, fmaf(-a0.y, h0.y, z0.x));
                z0.y = fmaf(a0.x, h0.y, fmaf(a0.y, h0.x, z0.y));
                z1.x = fmaf(a1.x, h1.x, fmaf(-a1.y, h1.y, z1.x));
                z1.y = fmaf(a1.x, h1.y, fmaf(a1.y, h1.x, z1.y));
            }
        }
        __syncthreads();
        // ---- I1: inverse radix-2, Ns = 1 ----
        dft2<true>(z0, z1);
        bufA[opad(2 * t)] = z0;
        bufA[opad(2 * t + 1)] = z1;
        __syncthreads();
        // ---- I2: inverse radix-8, Ns = 2 (A -> B), 128 lanes ----
        if (t < 128) {
            const int j = t, k = j & 1;
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = bufA[opad(j + 128 * r)];
            twiddle_tree<8>(v, conjf2(tw[256 * (jb & 1)]));
            Dft<8, true>::run(v);
            const int o = (j >> 1) * 16 + k;
#pragma unroll
            for (int r = 0; r < 8; ++r) bufB[opad(o + 2 * r)] = v[r];
        }
        __syncthreads();
        // ---- I3: inverse radix-8, Ns = 16 (B -> A) ----
        if (t < 128) {
            const int j = t, k = j & 15;
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = bufB[opad(j + 128 * r)];
            twiddle_tree<8>(v, conjf2(tw[32 * (jb & 15)]));
            Dft<8, true>::run(v);
            const int o = (j >> 4) * 128 + k;
#pragma unroll
            for (int r = 0; r < 8; ++r) bufA[opad(o + 16 * r)] = v[r];
        }
        __syncthreads();
        // ---- I4: inverse radix-8, Ns = 128 -> outputs i = j + 128 r ----
        if (t < 128) {
            const int j = t;
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = bufA[opad(j + 128 * r)];
            twiddle_tree<8>(v, conjf2(tw[4 * jb]));
            Dft<8, true>::run(v);
            const long m0 = q * p.M - skip + j;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int i = j + 128 * r;
                if (i >= skip && m0 + 128 * r < p.n_out) out[m0 + 128 * r] = v[r];
            }
        }
        __syncthreads();
    }

    if (blockIdx.x == gridDim.x - 1) {
        float2* hn = p.hist_next + ch * (long)(K - 1);
        for (int jj = t0; jj < K - 1; jj += kOs4Block) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

struct OsState {
    int D = 1, L = 4096, M = 0, K = 1;
    float2* d_H = nullptr;
    float2* d_tw = nullptr;
};

// ---------------------------------------------------------------------------------
// v5 (D = 4): three workgroup barriers per window, wave-local inverse FFTs.
//
// Forward, per window (4 branches x 1024 points, 256 lanes x 16 points):
//   branch element j = 64 n1 + n2, bin k = k1 + 16 k2, k2 = j1 + 16 j2, n2 = 4 m1 + m2
//   P1  lane t (n2 = t/4, branch 3 - t%4): 16-pt DFT over n1 of its 16 coalesced samples,
//       x W1024^(n2 k1) (per-lane constant twiddles), -> LDS A[b][k1][n2]         | barrier
//   P2  wave b, lane (k1, m2): 16-pt DFT over m1 of A[b][k1][4 m1 + m2], x W64^(m2 j1)
//       -> LDS B[b][m2][k1 + 16 j1] (wave-local: this wave's branch only)        | barrier
//   P3  lane kappa = k1 + 16 j1: 4-pt DFT over m2 per branch -> X_b[kappa + 256 j2],
//       Y = sum_b H_b X_b with H held in registers -> spectrum slot w (LDS)       | barrier
// Inverse, every 4 windows, wave v on slot v (64 lanes x 16 points, no barriers):
//   k = 64 k1 + k2, n = n1 + 16 n2, k2 = 16 c + a, n2 = d + 4 e
//   I1  lane k2: 16-pt IDFT over k1, x W1024^-(n1 k2)            -> E1[n1][k2]
//   I2  lane (a, n1 = l/16 + 4 i): 4-pt IDFT over c, x W64^-(d a)  -> E2[n1][d][a]
//   I3  lane n1 + 16 d: 16-pt IDFT over a -> y[lane + 64 e]: coalesced stores
// The next window's samples are loaded into the registers P1 has just consumed, so they
// stream in during P2, P3 and the inverse.  LDS: workspace 4 x 1092 + 4 spectrum slots x
// 1280 float2 = 75 KiB (2 workgroups per CU).
constexpr int kOs5Slot = 1280;
constexpr int kOs5Br = 1092;   // branch stride (== 4 mod 16)

__global__ __launch_bounds__(kOsBlock, 2) void fir_os5_kernel(OsParams p, long nblk) {
    constexpr int D = 4, L = 1024;
    __shared__ float2 ws[4 * kOs5Br];
    __shared__ float2 slots[4 * kOs5Slot];
    __shared__ float2 t64[64];  // W64^(m2 j1) at [16 m2 + j1]

    const long ch = blockIdx.y;
    const float2* __restrict__ in = p.in + ch * p.ld_in;
    const float2* __restrict__ hist = p.hist + ch * (long)(p.K - 1);
    float2* __restrict__ out = p.out + ch * p.ld_out;
    const float2* __restrict__ tw = p.tw;  // W4096^m
    const int K = p.K;
    const int skip = L - p.M;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;

    // ---- per-lane constants ----
    float2 w1[16], wi2[4];
    const float2 wi1b = conjf2(tw[(4 * lane) & 4095]);  // W1024^-(k2), k2 = lane
    if (t < 64) t64[t] = tw[(64 * (t >> 4) * (t & 15)) & 4095];
    {
        const int n2 = t >> 2;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            w1[r] = tw[(4 * n2 * r) & 4095];                 // W1024^(n2 r)
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) wi2[d] = conjf2(tw[(64 * d * (lane & 15)) & 4095]);  // W64^-(d a)
    }
    float2 H[4][4];  // H[b][j2] = H_b[kappa + 256 j2], kappa = t
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int j2 = 0; j2 < 4; ++j2) H[b][j2] = p.H[b * L + t + 256 * j2];

    const long nquad = (nblk + 3) / 4;
    float2 v[16];
    long quad = blockIdx.x;
    auto base_of = [&](long q) { return p.i0 + (q * p.M + p.M - L) * (long)D - (D - 1); };
    if (quad < nquad) os2_load<D>(v, in, hist, p.n_in, K, base_of(4 * quad) + t);

#pragma unroll 1
    for (; quad < nquad; quad += gridDim.x) {
#pragma unroll 1
        for (int w = 0; w < 4; ++w) {
            const long q = 4 * quad + w;
            // ---- P1 ----
            Dft<16, false>::run(v);
            {
                const int n2 = t >> 2, b = 3 - (t & 3);
                float2* dst = ws + b * kOs5Br + n2;
                dst[0] = v[0];
#pragma unroll
                for (int k1 = 1; k1 < 16; ++k1) dst[68 * k1] = cmul(v[k1], w1[k1]);
            }
            // ---- next window's samples fly during P2 / P3 / inverse ----
            {
                const long qn = (w < 3) ? q + 1 : 4 * (quad + gridDim.x);
                if (qn < 4 * nquad) os2_load<D>(v, in, hist, p.n_in, K, base_of(qn) + t);
            }
            __syncthreads();
            // ---- P2 (wave-local: wave = branch) ----
            {
                const int k1 = lane >> 2, m2 = lane & 3;
                float2* rb = ws + wave * kOs5Br + 68 * k1 + m2;
                float2 u[16];
#pragma unroll
                for (int m1 = 0; m1 < 16; ++m1) u[m1] = rb[4 * m1];
                Dft<16, false>::run(u);
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                float2* wb = ws + wave * kOs5Br + 260 * m2 + k1;
                const float2* tr = t64 + 16 * m2;
                wb[0] = u[0];
#pragma unroll
                for (int j1 = 1; j1 < 16; ++j1) wb[16 * j1] = cmul(u[j1], tr[j1]);
            }
            __syncthreads();
            // ---- P3: 4-pt DFTs, multiply by H, sum over branches ----
            {
                float2 y[4];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const float2* rb = ws + b * kOs5Br + t;
                    float2 a0 = rb[0], a1 = rb[260], a2 = rb[520], a3 = rb[780];
                    dft4<false>(a0, a1, a2, a3);
                    if (b == 0) {
                        y[0] = cmul(a0, H[0][0]);
                        y[1] = cmul(a1, H[0][1]);
                        y[2] = cmul(a2, H[0][2]);
                        y[3] = cmul(a3, H[0][3]);
                    } else {
                        const float2 x4[4] = {a0, a1, a2, a3};
#pragma unroll
                        for (int j2 = 0; j2 < 4; ++j2) {
                            y[j2].x = fmaf(x4[j2].x, H[b][j2].x, fmaf(-x4[j2].y, H[b][j2].y, y[j2].x));
                            y[j2].y = fmaf(x4[j2].x, H[b][j2].y, fmaf(x4[j2].y, H[b][j2].x, y[j2].y));
                        }
                    }
                }
                float2* sl = slots + w * kOs5Slot + t;
#pragma unroll
                for (int j2 = 0; j2 < 4; ++j2) sl[256 * j2] = y[j2];
            }
            __syncthreads();
        }

        // ---- inverse: wave v transforms slot v (window 4 quad + v) ----
        {
            const long q = 4 * quad + wave;
            float2* sl = slots + wave * kOs5Slot;
            float2 u[16];
            // I1: lane = k2
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) u[k1] = sl[64 * k1 + lane];
            Dft<16, true>::run(u);
            {
                // x W1024^-(n1 k2): powers of the lane's base (once per 4 windows)
                float2 wb = wi1b;
                asm volatile("" : "+v"(wb.x), "+v"(wb.y));
                twiddle_tree<16>(u, wb);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int n1 = 0; n1 < 16; ++n1) sl[80 * n1 + lane] = u[n1];
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            // I2: lane (a, n1 = lane/16 + 4 i)
            const int a = lane & 15, nb = lane >> 4;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 4; ++c) u[4 * i + c] = sl[80 * (nb + 4 * i) + 16 * c + a];
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dft4<true>(u[4 * i], u[4 * i + 1], u[4 * i + 2], u[4 * i + 3]);
                float2* wr = sl + 65 * (nb + 4 * i) + a;
                wr[0] = u[4 * i];
#pragma unroll
                for (int d = 1; d < 4; ++d) wr[16 * d] = cmul(u[4 * i + d], wi2[d]);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            // I3: lane = n1 + 16 d
            {
                const int n1 = lane & 15, d = lane >> 4;
#pragma unroll
                for (int aa = 0; aa < 16; ++aa) u[aa] = sl[65 * n1 + 16 * d + aa];
            }
            Dft<16, true>::run(u);
            if (q < nblk) {
                const long m0 = q * p.M - skip + lane;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int n = lane + 64 * e;
                    if (n >= skip && m0 + 64 * e < p.n_out) out[m0 + 64 * e] = u[e];
                }
            }
        }
        // slots are rewritten by the next quad's P3 only after two more barriers
    }

    if (blockIdx.x == gridDim.x - 1) {  // stream history carry (see fir_direct.hip)
        float2* hn = p.hist_next + ch * (long)(K - 1);
        for (int jj = t; jj < K - 1; jj += kOsBlock) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

int os_geometry(int K, int D, int* L, int* M) {
    if (!(D == 1 || D == 2 || D == 4 || D == 8)) return 0;
    const int l = kOsPoints / D;
    const int T = (K + D - 1) / D;
    const int skip = ((T - 1) + 31) / 32 * 32;
    if (T - 1 > l / 4) return 0;
    if (L) *L = l;
    if (M) *M = l - (skip > 0 ? skip : 0);
    return 1;
}

}  // namespace

int fir_os_supported(int sample_kind, int tap_kind, int K, int D) {
    (void)tap_kind;
    if (sample_kind != SDRGPU_C64) return 0;
    if (K < 2) return 0;
    return os_geometry(K, D, nullptr, nullptr);
}

void* fir_os_prepare(int device, int sample_kind, int tap_kind, const void* taps, int K, int D,
                     hipStream_t s, int* status) {
    (void)device;
    (void)s;
    if (!fir_os_supported(sample_kind, tap_kind, K, D)) {
        if (status) *status = SDRGPU_ERR_UNSUPPORTED;
        return nullptr;
    }
    auto* st = new OsState();
    st->D = D;
    st->K = K;
    os_geometry(K, D, &st->L, &st->M);
    const int L = st->L;
    // Branch spectra in float64: H_b[k] = (1/L) sum_i h[b + iD] exp(-2 pi i i k / L)
    std::vector<float2> H((size_t)D * L);
    std::vector<double> hr(K), hi(K, 0.0);
    for (int k = 0; k < K; ++k) {
        if (tap_kind == SDRGPU_C64) {
            hr[k] = static_cast<const float*>(taps)[2 * k];
            hi[k] = static_cast<const float*>(taps)[2 * k + 1];
        } else {
            hr[k] = static_cast<const float*>(taps)[k];
        }
    }
    for (int b = 0; b < D; ++b) {
        for (int k = 0; k < L; ++k) {
            double sr = 0.0, si = 0.0;
            for (int i = 0; b + i * D < K; ++i) {
                const long e = ((long)i * k) % L;
                const double a = -2.0 * M_PI * (double)e / (double)L;
                const double c = std::cos(a), sn = std::sin(a);
                const int q = b + i * D;
                sr += hr[q] * c - hi[q] * sn;
                si += hr[q] * sn + hi[q] * c;
            }
            H[(size_t)b * L + k] = make_float2((float)(sr / L), (float)(si / L));
        }
    }
    std::vector<float2> tw(kOsPoints);
    for (int m = 0; m < kOsPoints; ++m) {
        const double a = -2.0 * M_PI * (double)m / (double)kOsPoints;
        tw[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    if (hipMalloc(&st->d_H, H.size() * sizeof(float2)) != hipSuccess ||
        hipMalloc(&st->d_tw, tw.size() * sizeof(float2)) != hipSuccess ||
        hipMemcpy(st->d_H, H.data(), H.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(st->d_tw, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) {
        if (st->d_H) (void)hipFree(st->d_H);
        if (st->d_tw) (void)hipFree(st->d_tw);
        delete st;
        if (status) *status = SDRGPU_ERR_NOMEM;
        return nullptr;
    }
    if (status) *status = SDRGPU_OK;
    return st;
}

int fir_os_launch(const FirParams& fp, void* os_state, hipStream_t s) {
    auto* st = static_cast<OsState*>(os_state);
    if (!st || fp.sample_kind != SDRGPU_C64 || fp.D != st->D || fp.K != st->K)
        return SDRGPU_ERR_UNSUPPORTED;
    OsParams p;
    p.in = static_cast<const float2*>(fp.in);
    p.ld_in = fp.ld_in;
    p.n_in = fp.n_in;
    p.hist = static_cast<const float2*>(fp.hist);
    p.hist_next = static_cast<float2*>(fp.hist_next);
    p.i0 = fp.i0;
    p.n_out = fp.n_out;
    p.K = fp.K;
    p.M = st->M;
    p.H = st->d_H;
    p.tw = st->d_tw;
    p.out = static_cast<float2*>(fp.out);
    p.ld_out = fp.ld_out;
    const long nblk = fp.n_out > 0 ? ceil_div(fp.n_out, st->M) : 1;
    dim3 grid((unsigned)nblk, (unsigned)fp.nch);
    // Kernel variants (debug/A-B knob SDRGPU_OS_VARIANT; all parity-tested), D = 4 | 8:
    //   11 (default) persistent v2, branch spectra in registers, 4 WG/CU
    //    1 persistent v2, spectra re-read from L2 every window      0 / 10 + next-window prefetch
    //    2 v1 (one window per workgroup)   3 / 4 two / one windows per iteration (v3)
    //    5 / 6 512-lane radix-8 (v4)       9 three-barrier, wave-local inverse (v5)
    //    7 / 8 ablations: memory only / FFT only (results invalid)
    //   12 = 11 at 3 WG/CU
    static const char* var_env = getenv("SDRGPU_OS_VARIANT");
    static const char* force_v1 = getenv("SDRGPU_OS_V1");
    int variant = var_env ? atoi(var_env) : 11;
    if (force_v1 && force_v1[0] == '1') variant = 2;
    const int wgs_per_cu = variant == 1 ? 4 : variant == 3 ? 2 : variant == 4 ? 4 : variant == 5 ? 4 : variant == 6 ? 3 : variant == 12 ? 3 : variant >= 7 ? 4 : 3;  // 11/12: H in registers at 4/3 WG per CU
    const long per_ch = std::max(1L, std::min(nblk, (256L * wgs_per_cu + fp.nch - 1) / fp.nch));
    const long per_ch2 = std::max(1L, std::min((nblk + 1) / 2, (256L * wgs_per_cu + fp.nch - 1) / fp.nch));
    dim3 pgrid2((unsigned)per_ch2, (unsigned)fp.nch);
    dim3 pgrid((unsigned)per_ch, (unsigned)fp.nch);
    switch (st->D) {
    case 1: hipLaunchKernelGGL(fir_os_kernel<1>, grid, dim3(kOsBlock), 0, s, p); break;
    case 2: hipLaunchKernelGGL(fir_os_kernel<2>, grid, dim3(kOsBlock), 0, s, p); break;
    case 4:
        if (variant == 0) hipLaunchKernelGGL((fir_os2_kernel<4, true, 3>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 1) hipLaunchKernelGGL((fir_os2_kernel<4, false, 4>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 3) hipLaunchKernelGGL((fir_os3_kernel<4, 2, 2>), pgrid2, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 4) hipLaunchKernelGGL((fir_os3_kernel<4, 1, 4>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 5) hipLaunchKernelGGL((fir_os4_kernel<8>), pgrid, dim3(kOs4Block), 0, s, p, nblk);
        else if (variant == 7) hipLaunchKernelGGL((fir_os3_kernel<4, 1, 4, 1>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 8) hipLaunchKernelGGL((fir_os3_kernel<4, 1, 4, 2>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 10) hipLaunchKernelGGL((fir_os2_kernel<4, true, 4>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 11) hipLaunchKernelGGL((fir_os2_kernel<4, false, 4, true>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 12) hipLaunchKernelGGL((fir_os2_kernel<4, false, 3, true>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 9) {
            const long nquad = (nblk + 3) / 4;
            dim3 g5((unsigned)std::max(1L, std::min(nquad, (256L * 2 + fp.nch - 1) / fp.nch)), (unsigned)fp.nch);
            hipLaunchKernelGGL(fir_os5_kernel, g5, dim3(kOsBlock), 0, s, p, nblk);
        }
        else if (variant == 6) hipLaunchKernelGGL((fir_os4_kernel<6>), pgrid, dim3(kOs4Block), 0, s, p, nblk);
        else hipLaunchKernelGGL(fir_os_kernel<4>, grid, dim3(kOsBlock), 0, s, p);
        break;
    case 8:
        if (variant == 0) hipLaunchKernelGGL((fir_os2_kernel<8, true, 3>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 1) hipLaunchKernelGGL((fir_os2_kernel<8, false, 4>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        else if (variant == 2) hipLaunchKernelGGL(fir_os_kernel<8>, grid, dim3(kOsBlock), 0, s, p);
        else hipLaunchKernelGGL((fir_os2_kernel<8, false, 4, true>), pgrid, dim3(kOsBlock), 0, s, p, nblk);
        break;
    default: return SDRGPU_ERR_UNSUPPORTED;
    }
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

void fir_os_release(void* os_state) {
    auto* st = static_cast<OsState*>(os_state);
    if (!st) return;
    if (st->d_H) (void)hipFree(st->d_H);
    if (st->d_tw) (void)hipFree(st->d_tw);
    delete st;
}

}  // namespace sdrgpu
