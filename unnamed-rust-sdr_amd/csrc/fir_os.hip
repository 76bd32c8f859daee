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
#include "fir_exact.hpp"

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
    int D, tpp, tap_c64;  // for fir_exact_output
    const void* taps_pm;
};

// an FFT block mixes every sample it holds, so one inf / NaN makes all of its outputs
// non-finite; a lane holding such outputs stores the reference's sum for them instead
// (fir_exact.hpp), outputs m0 + stride * r, r < n (those with ok(r))
template <typename OK>
__device__ __forceinline__ void os_exact(const OsParams& p, const float2* __restrict__ in,
                                                 const float2* __restrict__ hist,
                                                 float2* __restrict__ out, long m0, int stride,
                                                 int n, OK ok) {
#pragma unroll 1
    for (int r = 0; r < n; ++r) {
        const long m = m0 + (long)stride * r;
        if (!ok(r) || m >= p.n_out) continue;
        out[m] = p.tap_c64 ? fir_exact_output<float2, float2>(p, in, hist, m)
                           : fir_exact_output<float2, float>(p, in, hist, m);
    }
}

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
            bool bad = false;
#pragma unroll
            for (int r = 0; r < 16; ++r) bad |= !all_finite(v[r]);
            if (bad) {
                os_exact(p, in, hist, out, m0 + j - skip, NBI, 16, [&](int r) { return j + NBI * r >= skip; });
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = j + NBI * r;
                    const long m = m0 + (i - skip);
                    if (i >= skip && m < p.n_out) out[m] = v[r];
                }
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
            if (!((int)all_finite(a0) & (int)all_finite(a1) & (int)all_finite(a2) & (int)all_finite(a3))) {
                os_exact(p, in, hist, out, m0, NI, 4, [&](int r) { return j + NI * r >= skip; });
            } else {
                if (j >= skip && m0 < p.n_out) o[0] = a0;
                if (j + NI >= skip && m0 + NI < p.n_out) o[NI] = a1;
                if (j + 2 * NI >= skip && m0 + 2 * NI < p.n_out) o[2 * NI] = a2;
                if (j + 3 * NI >= skip && m0 + 3 * NI < p.n_out) o[3 * NI] = a3;
            }
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

struct OsState {
    int D = 1, L = 4096, M = 0, K = 1;
    float2* d_H = nullptr;
    float2* d_tw = nullptr;
};

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
    p.D = fp.D;
    p.tpp = fp.tpp;
    p.tap_c64 = fp.tap_kind == SDRGPU_C64;
    p.taps_pm = fp.taps_pm;
    const long nblk = fp.n_out > 0 ? ceil_div(fp.n_out, st->M) : 1;
    dim3 grid((unsigned)nblk, (unsigned)fp.nch);
    // D = 4 | 8: persistent workgroups (4 per CU) with the branch spectra in registers; the
    // round-1 A/B variants (prefetching, interleaved windows, 512-lane radix-8, three-barrier)
    // measured slower and were removed from the product
    const long per_ch = std::max(1L, std::min(nblk, (256L * 4 + fp.nch - 1) / fp.nch));
    dim3 pgrid((unsigned)per_ch, (unsigned)fp.nch);
    switch (st->D) {
    case 1: hipLaunchKernelGGL(fir_os_kernel<1>, grid, dim3(kOsBlock), 0, s, p); break;
    case 2: hipLaunchKernelGGL(fir_os_kernel<2>, grid, dim3(kOsBlock), 0, s, p); break;
    case 4: hipLaunchKernelGGL((fir_os2_kernel<4, false, 4, true>), pgrid, dim3(kOsBlock), 0, s, p, nblk); break;
    case 8: hipLaunchKernelGGL((fir_os2_kernel<8, false, 4, true>), pgrid, dim3(kOsBlock), 0, s, p, nblk); break;
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
