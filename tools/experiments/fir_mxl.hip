// fir_mxl.hip -- LDS-staged split-bf16 MFMA direct-form FIR, decimate by 4 (gfx950).
//
// Semantics: Fir::apply + Decimate (reference src/filter/fir.rs:23-32,
// src/filter/convolve.rs:13-15, src/signal/adapters/mod.rs:30-37) for complex samples and
// real taps: y[m] = sum_k h[k] x[i0 + 4m - k], zero history before the stream start.
//
// Arithmetic (as fir_mfma.hip): every f32 is split EXACTLY into three bf16 pieces
// (x = xh + xm + xl, truncation split) and x*h is formed from the six products
// xh*hh + xh*hm + xm*hh + xh*hl + xm*hm + xl*hh on v_mfma_f32_16x16x32_bf16 (dropped terms
// < 2^-21 |x h|; f32's exponent range is kept, so any input scale works).
//
// GEMM shape.  A wave owns a contiguous run of TILES of 256 kept outputs (1024 input
// samples).  A tile is C[16 x 16] += A[16 x 32] B[32 x 16] over NCH 32-sample chunks:
//   rows    u = output offset inside a 16-output block            (A = taps, registers)
//   columns v = one of the tile's 16 blocks of 16 outputs         (B = samples, LDS)
//   K       = the 32*NCH-sample window of block v (windows of consecutive blocks are
//             64 samples apart); A[u][p] = h[4u + 3 - delta + H - p] (banded Toeplitz;
//             NCH = 10 at K = 255, so 80 % of the MFMA work is useful).
// Why LDS: fir_mfma.hip feeds each lane's fragment straight from HBM (16 segments per
// wave-instruction, 64 B each) and that access pattern caps the stream at ~56 % of HBM.
// Here each wave streams ITS OWN contiguous range with 1 KiB-contiguous dwordx4 loads,
// splits every sample once into six bf16 planes (hi/mid/lo x re/im) in LDS, and each
// block window is read back as 16-byte B fragments: HBM sees every byte once, the 5x
// window overlap is served by LDS.
//
// LDS (wave-private, no barriers): per plane a ring of two tiles (2048 samples) plus an
// H-sample mirror of the ring's tail in front of it, so every window is contiguous.  Byte
// address of buffer sample b: 128*(b>>6) + 16*(((b>>3)&7) ^ ((b>>7)&7)) + 2*(b&7)
// (64-sample rows, 16-byte quads XOR-swizzled by row/2).  MFMA column v computes block
// sigma(v), which sends lanes {0-3,12-15} to even and {4-11} to odd blocks: every 16-lane
// group of a ds_read_b128 then reads 8 even and 8 odd rows with 8 distinct swizzle keys
// each -- conflict-free for every chunk; the ds_write_b32 staging is conflict-free too.
//
// Pipeline per tile t (tau = t & 1 picks the ring half, so all LDS offsets are
// immediates): read chunk c's six B fragments, 12 MFMAs; interleaved with them, split and
// write tile t+1's samples (already in registers) into the other ring half -- the groups
// that land on the history region tile t still reads go after the chunk that last reads
// it; LDS executes one wave's operations in order -- and reload the freed registers with
// tile t+3's samples (two tiles of latency cover).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "fir_kernels.hpp"

namespace sdrgpu {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kD = 4;
constexpr int kTileOut = 256;
constexpr int kTileIn = kTileOut * kD;  // 1024 new samples per tile
constexpr int kRing = 2 * kTileIn;
constexpr int kWaves = 4;               // one wave per SIMD
constexpr int kBlock = 64 * kWaves;

template <int NCH>
struct Geo {
    static constexpr int H = 32 * NCH - 16 * kD;    // history samples a tile's windows need
    static constexpr int BUF = kRing + H;           // samples per plane
    static constexpr int PLANE = 2 * BUF;           // bytes per plane (bf16)
    static constexpr int WAVE = 6 * PLANE;          // bytes per wave
    static constexpr int KM = (kTileIn - H) / 128;  // first 128-sample group on the history
    static constexpr int NH = H / 128;              // warm-up groups
    static_assert(H % 128 == 0 && H > 0 && H < kTileIn, "geometry");
};

struct MxlParams {
    const float2* in;
    long ld_in, n_in;
    const float2* hist;
    float2* hist_next;
    const float2* dummy;  // >= 1024 readable samples: target of clamped prefetches
    long n_out;
    int K;
    int delta;  // 3 - i0
    const float* taps;
    float2* out;
    long ld_out;
    long tpc;        // tiles per channel
    long spc;        // segments per channel
    long seg_tiles;  // tiles per segment
    long units;      // nch * spc
    int vec_out;     // 16-byte output stores allowed
};

__device__ __forceinline__ void split3(float a, float b, unsigned& hi, unsigned& mid,
                                       unsigned& lo) {
    const unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
    hi = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
    const float ra = a - __uint_as_float(ua & 0xffff0000u);
    const float rb = b - __uint_as_float(ub & 0xffff0000u);
    const unsigned ura = __float_as_uint(ra), urb = __float_as_uint(rb);
    mid = __builtin_amdgcn_perm(urb, ura, 0x07060302u);
    const float la = ra - __uint_as_float(ura & 0xffff0000u);
    const float lb = rb - __uint_as_float(urb & 0xffff0000u);
    lo = __builtin_amdgcn_perm(__float_as_uint(lb), __float_as_uint(la), 0x07060302u);
}

__device__ __forceinline__ f32x4 mfma(const u32x4& a, const u32x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// block of the tile that MFMA column v computes (header: even/odd split of the lanes)
__device__ __forceinline__ int sigma(int v) {
    return v < 4 ? 2 * v : (v >= 12 ? 2 * v - 16 : 2 * v - 7);
}

__device__ __forceinline__ float2 fetch1(const float2* in, const float2* hist, long j, long n_in,
                                         int K) {
    const bool inb = (j >= 0) & (j < n_in);
    const bool inh = (j < 0) & (j >= -(long)(K - 1));
    const float2 xa = in[inb ? j : 0];
    const float2 xb = hist[inh ? j + (K - 1) : 0];
    return inb ? xa : (inh ? xb : make_float2(0.f, 0.f));
}

// sample pair (j, j+1) with history / zero fill (slow path: stream start and end)
__device__ __forceinline__ float4 fetch_pair(const float2* in, const float2* hist, long j,
                                             long n_in, int K) {
    const float2 a = fetch1(in, hist, j, n_in, K), b = fetch1(in, hist, j + 1, n_in, K);
    return make_float4(a.x, a.y, b.x, b.y);
}

__device__ __forceinline__ void st32(char* lds, int a, unsigned v) {
    *reinterpret_cast<unsigned*>(lds + a) = v;
}

// split one sample pair into the six planes at byte offset a (+ immediate plane offsets)
template <int PLANE>
__device__ __forceinline__ void put_pair(char* lds, int a, const float4& f) {
    unsigned h, m, l;
    split3(f.x, f.z, h, m, l);
    st32(lds, a, h);
    st32(lds, a + PLANE, m);
    st32(lds, a + 2 * PLANE, l);
    split3(f.y, f.w, h, m, l);
    st32(lds, a + 3 * PLANE, h);
    st32(lds, a + 4 * PLANE, m);
    st32(lds, a + 5 * PLANE, l);
}

// chunk after whose B reads group k of the next tile is staged
template <int NCH>
constexpr int stage_slot(int k) {
    using G = Geo<NCH>;
    return k < G::KM ? (k < NCH - 1 ? k : NCH - 1)
                     : (G::H / 32 + (k - G::KM) < NCH - 1 ? G::H / 32 + (k - G::KM) : NCH - 1);
}

// ABL (debug ablation, results invalid): 1 = memory only (no LDS reads / MFMA),
// 2 = no HBM loads (compute only)
template <int NCH, int ABL = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fir_mxl_kernel(MxlParams p) {
    using G = Geo<NCH>;
    constexpr int H = G::H, PL = G::PLANE, KM = G::KM;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const long wave = (long)blockIdx.x * kWaves + wv;
    const long nwaves = (long)gridDim.x * kWaves;
    const int g = lane >> 4, v = lane & 15;
    const int K = p.K;
    const int base = wv * G::WAVE;

    // ---- A: tap Toeplitz fragments, A[u = lane % 16][p = 32c + 8g + j] ----
    u32x4 ah[NCH], am[NCH], al[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            float hv[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int pidx = 32 * c + 8 * g + 2 * jj + e;
                const int k = 4 * v + 3 - p.delta + H - pidx;
                const bool ok = (k >= 0) & (k < K);
                const float hk = p.taps[ok ? k : 0];
                hv[e] = ok ? hk : 0.f;
            }
            unsigned h, m, l;
            split3(hv[0], hv[1], h, m, l);
            ah[c][jj] = h;
            am[c][jj] = m;
            al[c][jj] = l;
        }
    }

    // ---- LDS address maps (bytes) ----
    const int sv = sigma(v);
    int rb[NCH];  // B fragment of chunk c in ring half 0
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int r = sv + (c >> 1);
        rb[c] = base + 128 * r + 16 * ((4 * (c & 1) + g) ^ ((r >> 1) & 7));
    }
    // sample pair (2 lane, 2 lane + 1) of a 128-sample group: rows 2k + lane/32
    const int wb0 = base + 128 * (lane >> 5) + 4 * (lane & 3) + 16 * ((lane >> 2) & 7);

    for (long u = wave; u < p.units; u += nwaves) {
        const long ch = u / p.spc;
        const long t0 = (u - ch * p.spc) * p.seg_tiles;
        const long nt = std::min(p.seg_tiles, p.tpc - t0);
        if (nt <= 0) continue;
        const float2* __restrict__ in = p.in + ch * p.ld_in;
        const float2* __restrict__ hist = p.hist + ch * (long)(K - 1);
        float2* __restrict__ out = p.out + ch * p.ld_out;
        const long n_in = p.n_in;
        const long N0 = (long)kTileIn * t0;   // first new sample of the segment's tile 0
        long ntf = (n_in - N0) / kTileIn;     // tiles entirely inside [0, n_in)
        ntf = n_in < N0 ? 0 : (ntf > nt ? nt : ntf);

        auto load_tile = [&](float4 (&dst)[8], long t) {
            const long j0 = N0 + (long)kTileIn * t;
            if (ABL == 2) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    dst[k] = make_float4((float)(j0 + k), 1.f, 2.f, (float)lane);
                return;
            }
            if (t < ntf) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    dst[k] = *reinterpret_cast<const float4*>(in + j0 + 128 * k + 2 * lane);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    dst[k] = fetch_pair(in, hist, j0 + 128 * k + 2 * lane, n_in, K);
            }
        };

        float4 ra[8], rn[8];
        {   // warm-up: the H samples before tile 0 -> mirror region [0, H)
            float4 wu[G::NH];
#pragma unroll
            for (int k = 0; k < G::NH; ++k)
                wu[k] = fetch_pair(in, hist, N0 - H + 128 * k + 2 * lane, n_in, K);
#pragma unroll
            for (int k = 0; k < G::NH; ++k)
                put_pair<PL>(smem, (wb0 ^ (16 * (k & 7))) + 256 * k, wu[k]);
        }
        load_tile(ra, 0);
        if (nt > 1) load_tile(rn, 1);
#pragma unroll
        for (int k = 0; k < 8; ++k)  // tile 0 -> ring half 0
            put_pair<PL>(smem, (wb0 ^ (16 * ((H / 128 + k) & 7))) + 128 * (H / 64 + 2 * k),
                         ra[k]);
        if (nt > 2) load_tile(ra, 2);

        // compute tile t (ring half TAU) while staging tile t+1 from `nx` (half 1 - TAU)
        auto body = [&](auto tau_c, long t, float4 (&nx)[8]) {
            constexpr int TAU = decltype(tau_c)::value;
            constexpr int TN = 1 - TAU;
            const bool fast3 = t + 3 < ntf;
            const float2* src3 = fast3 ? in + N0 + (long)kTileIn * (t + 3) : p.dummy;
            f32x4 cr = {0.f, 0.f, 0.f, 0.f}, ci = {0.f, 0.f, 0.f, 0.f};
            // B fragments of chunk c are read one chunk ahead of their MFMAs
            u32x4 fb[2][6];
            auto read_frags = [&](u32x4 (&f)[6], int c) {
                const int a = rb[c] + 2048 * TAU;
#pragma unroll
                for (int q = 0; q < 6; ++q)
                    f[q] = *reinterpret_cast<const u32x4*>(smem + a + q * PL);
            };
            if (ABL != 1) read_frags(fb[0], 0);
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                if (ABL != 1) {
                    if (c + 1 < NCH) read_frags(fb[(c + 1) & 1], c + 1);
                    // keep the next chunk's reads ahead of this chunk's MFMAs (the machine
                    // scheduler would otherwise sink them next to their first use)
                    __builtin_amdgcn_sched_barrier(0);
                    const u32x4(&f)[6] = fb[c & 1];
                    const u32x4 rh = f[0], rm = f[1], rl = f[2], ih = f[3], im = f[4], il = f[5];
                    cr = mfma(al[c], rh, cr);
                    ci = mfma(al[c], ih, ci);
                    cr = mfma(am[c], rm, cr);
                    ci = mfma(am[c], im, ci);
                    cr = mfma(ah[c], rl, cr);
                    ci = mfma(ah[c], il, ci);
                    cr = mfma(am[c], rh, cr);
                    ci = mfma(am[c], ih, ci);
                    cr = mfma(ah[c], rm, cr);
                    ci = mfma(ah[c], im, ci);
                    cr = mfma(ah[c], rh, cr);
                    ci = mfma(ah[c], ih, ci);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (stage_slot<NCH>(k) != c) continue;
                    put_pair<PL>(smem,
                                 (wb0 ^ (16 * ((H / 128 + k) & 7))) + 2048 * TN +
                                     128 * (H / 64 + 2 * k),
                                 nx[k]);
                    if (TN == 1 && k >= KM)  // ring tail -> its mirror in front
                        put_pair<PL>(smem, (wb0 ^ (16 * ((k - KM) & 7))) + 256 * (k - KM), nx[k]);
                    if (ABL != 2)
                        nx[k] = *reinterpret_cast<const float4*>(src3 + 128 * k + 2 * lane);
                }
            }
            // tile t+3 not entirely inside the input (channel end): guarded reload
            if (!fast3 && t + 3 < nt) load_tile(nx, t + 3);
            // ---- store tile t: the lane holds outputs 16 sigma(v) + 4g + i ----
            const long m = (t0 + t) * kTileOut + 16 * sv + 4 * g;
            if (p.vec_out && (t0 + t + 1) * kTileOut <= p.n_out) {
                *reinterpret_cast<float4*>(out + m) = make_float4(cr[0], ci[0], cr[1], ci[1]);
                *reinterpret_cast<float4*>(out + m + 2) = make_float4(cr[2], ci[2], cr[3], ci[3]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (m + i < p.n_out) out[m + i] = make_float2(cr[i], ci[i]);
            }
        };

        for (long t = 0; t < nt; t += 2) {
            body(std::integral_constant<int, 0>(), t, rn);
            if (t + 1 >= nt) break;
            body(std::integral_constant<int, 1>(), t + 1, ra);
        }
    }

    if (p.hist_next) {  // stream history carry, spread over the whole grid
        const long nch = p.units / p.spc;
        for (long j = (long)blockIdx.x * kBlock + threadIdx.x; j < nch * (K - 1);
             j += (long)gridDim.x * kBlock) {
            const long ch = j / (K - 1), jj = j - ch * (K - 1);
            const float2* inc = p.in + ch * p.ld_in;
            const float2* hic = p.hist + ch * (long)(K - 1);
            const long gidx = p.n_in - (long)(K - 1) + jj;
            p.hist_next[j] = gidx >= 0 ? inc[gidx] : hic[gidx + (K - 1)];
        }
    }
}

int mxl_nch(int K) {
    const int need = (K + 63 + 31) / 32;  // 32 NCH >= K + 15*4 + 3
    if (need <= 6) return 6;
    if (need <= 10) return 10;
    if (need <= 14) return 14;
    return 0;
}

}  // namespace

int fir_mxl_supported(const FirParams& fp) {
    if (fp.sample_kind != SDRGPU_C64 || fp.tap_kind != SDRGPU_F32 || fp.D != kD) return 0;
    if (fp.K < 1 || mxl_nch(fp.K) == 0) return 0;
    if (fp.i0 < 0 || fp.i0 >= kD) return 0;
    if ((reinterpret_cast<uintptr_t>(fp.in) & 15) != 0 || (fp.nch > 1 && (fp.ld_in & 1)))
        return 0;
    return 1;
}

size_t fir_mxl_dummy_bytes() { return (size_t)kTileIn * sizeof(float2); }

int fir_mxl_launch(const FirParams& fp, const float* d_taps, const void* d_dummy, int cus,
                   hipStream_t s) {
    if (!fir_mxl_supported(fp) || !d_dummy) return SDRGPU_ERR_UNSUPPORTED;
    const int NCH = mxl_nch(fp.K);
    MxlParams p;
    p.in = static_cast<const float2*>(fp.in);
    p.ld_in = fp.ld_in;
    p.n_in = fp.n_in;
    p.hist = static_cast<const float2*>(fp.hist);
    p.hist_next = fp.K > 1 ? static_cast<float2*>(fp.hist_next) : nullptr;
    p.dummy = static_cast<const float2*>(d_dummy);
    p.n_out = fp.n_out;
    p.K = fp.K;
    p.delta = (int)(kD - 1 - fp.i0);
    p.taps = d_taps;
    p.out = static_cast<float2*>(fp.out);
    p.ld_out = fp.ld_out;
    p.vec_out = ((reinterpret_cast<uintptr_t>(fp.out) & 15) == 0 &&
                 (fp.nch == 1 || !(fp.ld_out & 1)))
                    ? 1
                    : 0;
    const long nch = fp.nch;
    p.tpc = ceil_div(std::max(0L, fp.n_out), kTileOut);
    const long W = (long)kWaves * cus;
    long spc = nch >= W ? 1 : ceil_div(W, nch);
    spc = std::max(1L, std::min(spc, p.tpc));
    p.seg_tiles = std::max(1L, ceil_div(p.tpc, spc));
    static const long seg_env = [] {
        const char* e = getenv("SDRGPU_MXL_SEG");
        return e ? atol(e) : 0L;
    }();
    if (seg_env > 0) p.seg_tiles = std::min(p.seg_tiles, seg_env);
    p.spc = std::max(1L, ceil_div(p.tpc, p.seg_tiles));
    p.units = nch * p.spc;
    const long blocks = std::max(1L, std::min((long)cus, ceil_div(p.units, kWaves)));
    static const char* abl_env = getenv("SDRGPU_MX_ABLATION");
    const int abl = abl_env ? atoi(abl_env) : 0;
#define SDRGPU_MXL_CASE(CC)                                                                    \
    if (NCH == CC) {                                                                           \
        const size_t lds = (size_t)kWaves * Geo<CC>::WAVE;                                     \
        if (abl == 1)                                                                          \
            hipLaunchKernelGGL((fir_mxl_kernel<CC, 1>), dim3(blocks), dim3(kBlock), lds, s, p); \
        else if (abl == 2)                                                                     \
            hipLaunchKernelGGL((fir_mxl_kernel<CC, 2>), dim3(blocks), dim3(kBlock), lds, s, p); \
        else                                                                                   \
            hipLaunchKernelGGL((fir_mxl_kernel<CC, 0>), dim3(blocks), dim3(kBlock), lds, s, p); \
        SDRGPU_LAUNCH_CHECK();                                                                 \
        return SDRGPU_OK;                                                                      \
    }
    SDRGPU_MXL_CASE(10)
    SDRGPU_MXL_CASE(6)
    SDRGPU_MXL_CASE(14)
#undef SDRGPU_MXL_CASE
    return SDRGPU_ERR_UNSUPPORTED;
}

}  // namespace sdrgpu
