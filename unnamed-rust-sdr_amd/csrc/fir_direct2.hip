// fir_direct2.hip -- wave-private, persistent direct-form FIR / FIR-decimate for c64
// samples and f32 taps (the BASELINE configs[1] shape: 255 taps, D = 4).
//
// Semantics as fir_direct.hip (Fir::apply + Decimate, src/filter/fir.rs:23-32,
// src/signal/adapters/mod.rs:30-37): y[m] = sum_k h[k] x[g_m - k], g_m = i0 + m*D.
//
// Why direct form on gfx950: one complex-sample x real-tap MAC is exactly one
// v_pk_fma_f32 (acc.xy += x.xy * h.xx, h an SGPR pair with op_sel), so the whole FIR is
// 2^26 x 255 packed FMAs for configs[1] -- about half the HBM time of the same launch at
// VALU peak, and no FFT round trips through LDS.  The kernel is built so that nothing but
// those FMAs and one LDS read per R of them sits in the inner loop:
//
//  * a TILE is 64 lanes x R consecutive kept outputs; its input span (SPAN = D*R samples per
//    lane + a history halo of H = D*tpp samples) lives in a WAVE-PRIVATE LDS region, so no
//    workgroup barrier is ever needed (LDS ops of one wave execute in order);
//  * LDS layout: sample s at s + s/SPAN (one pad per lane span).  Lane t's window starts at
//    H + SPAN*t, so every read offset is a compile-time constant from the lane base, and
//    lanes are (SPAN+1) samples = 2*SPAN+2 dwords apart -> conflict-free ds_read_b64;
//  * polyphase: tap k = D*a + p.  For phase p the R outputs of a lane read the window
//    X_p[e] = x[base + D*e - p], e = j - a; stepping a slides the window by one, so each
//    ds_read_b64 feeds R packed FMAs (taps are wave-uniform scalar loads);
//  * persistent waves: while a tile is computed, the next tile's samples are already in
//    flight into registers (NL loads per lane), so HBM streaming overlaps the FMAs.
//
// Roofline: HBM bound at 8 B in (+ halo re-read from L2) + 8/D B out per input sample.
#include <algorithm>
#include <cstdlib>

#include "fir_exact.hpp"

namespace sdrgpu {

namespace {

constexpr int kD2Block = 256;  // 4 waves, each on its own tiles
constexpr int kD2Chunk = 16;   // taps per unrolled chunk (tpp is padded to a multiple)

template <int D> struct D2Geom {
    static constexpr int R = D == 1 ? 16 : D == 2 ? 16 : D == 4 ? 8 : 4;
    static constexpr int SPAN = D * R;  // input samples per lane per tile
    static_assert((D * kD2Chunk) % SPAN == 0, "chunk shift must be a whole number of spans");
};

// padded LDS offset of a (possibly negative) sample offset relative to a span boundary
template <int SPAN>
__host__ __device__ constexpr int d2pad(int s) {
    return s + (s >= 0 ? s / SPAN : -((-s + SPAN - 1) / SPAN));
}

__device__ __forceinline__ float2 fetch_c64(const float2* __restrict__ in, long n_in,
                                            const float2* __restrict__ hist, int K, long g) {
    if (g >= 0) return g < n_in ? in[g] : make_float2(0.f, 0.f);
    if (g >= -(long)(K - 1)) return hist[g + (K - 1)];
    return make_float2(0.f, 0.f);
}

template <int D, int NL>
__global__ __launch_bounds__(kD2Block, 2) void fir_direct2_kernel(FirParams p, long ntiles,
                                                                  int wave_lds) {
    using G = D2Geom<D>;
    constexpr int R = G::R, SPAN = G::SPAN, C = kD2Chunk;
    extern __shared__ __align__(16) unsigned char smem_raw[];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float2* const wl = reinterpret_cast<float2*>(smem_raw) + wave * wave_lds;

    const long ch = blockIdx.y;
    const float2* __restrict__ in = static_cast<const float2*>(p.in) + ch * p.ld_in;
    const float2* __restrict__ hist = static_cast<const float2*>(p.hist) + ch * (long)(p.K - 1);
    float2* __restrict__ out = static_cast<float2*>(p.out) + ch * p.ld_out;
    // constant address space: wave-uniform tap reads become s_load (lgkmcnt), never vector
    // loads that would share vmcnt with the in-flight next-tile prefetch
    using cfloat = const __attribute__((address_space(4))) float;
    cfloat* taps = (cfloat*)(p.taps_pm);
    const int K = p.K;
    const int tpp = p.tpp;
    const int H = D * tpp;                 // halo (multiple of SPAN)
    const int nchunk = tpp / C;
    constexpr long TO = 64L * R;           // kept outputs per tile

    // staging of one tile: lane loads samples lane + 64 i, i < NL.  Interior tiles are
    // prefetched into registers; tiles touching the stream edges (history / end) are
    // fetched element-wise straight into LDS at store time instead.
    float2 st[NL];
    auto tile_s0 = [&](long tile) { return p.i0 + tile * TO * D - H; };
    auto interior = [&](long s0) { return s0 >= 0 && s0 + 64L * NL <= p.n_in; };
    auto load_tile = [&](long tile) {
        const long s0 = tile_s0(tile);
        if (interior(s0)) {
            const float2* src = in + s0 + lane;
#pragma unroll
            for (int i = 0; i < NL; ++i) st[i] = src[64 * i];
        }
    };

    long tile = (long)blockIdx.x * (kD2Block / 64) + wave;
    const long tstride = (long)gridDim.x * (kD2Block / 64);
    if (tile < ntiles) load_tile(tile);

    // lane's padded window base: d2pad(H + SPAN*lane) = H + H/SPAN + (SPAN+1)*lane
    const int wbase = H + H / SPAN + (SPAN + 1) * lane;
    // staging store offsets: sample lane + 64 i -> padded
    const int sbase = lane + lane / SPAN;

#pragma unroll 1
    for (; tile < ntiles; tile += tstride) {
        // ---- staged samples -> wave-private LDS (WAR vs the previous tile's reads is
        // ordered: LDS ops of one wave complete in issue order) ----
        {
            const long s0 = tile_s0(tile);
            if (interior(s0)) {
#pragma unroll
                for (int i = 0; i < NL; ++i) wl[sbase + 64 * i + 64 * i / SPAN] = st[i];
            } else {
#pragma unroll 1
                for (int i = 0; i < NL; ++i)
                    wl[sbase + 64 * i + 64 * i / SPAN] = fetch_c64(in, p.n_in, hist, K, s0 + lane + 64 * i);
            }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        // ---- next tile's samples start flying ----
        if (tile + tstride < ntiles) load_tile(tile + tstride);

        float2 acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = make_float2(0.f, 0.f);

        const float2* const lb = wl + wbase;
#pragma unroll
        for (int ph = 0; ph < D; ++ph) {
            cfloat* hp = taps + ph * tpp;
            // window carry: cur[e-1] = X_p[e], e = 1..R-1 (chunk-relative)
            float2 cur[R > 1 ? R - 1 : 1];
#pragma unroll
            for (int e = 1; e < R; ++e) cur[e - 1] = lb[d2pad<SPAN>(D * e - ph)];
#pragma unroll 1
            for (int c = 0; c < nchunk; ++c) {
                // chunk c shifts the window by C taps = D*C samples = (D*C/SPAN) spans
                const float2* lc = lb - c * (D * C / SPAN) * (SPAN + 1);
                float2 nw[C];  // nw[i] = X_p[-i]
#pragma unroll
                for (int i = 0; i < C; ++i) nw[i] = lc[d2pad<SPAN>(-D * i - ph)];
                cfloat* hc = hp + c * C;
#pragma unroll
                for (int i = 0; i < C; ++i) {
                    const float h = hc[i];
#pragma unroll
                    for (int j = 0; j < R; ++j) {
                        const int e = j - i;
                        const float2 x = e >= 1 ? cur[e - 1] : nw[-e];
                        acc[j].x = fmaf(x.x, h, acc[j].x);
                        acc[j].y = fmaf(x.y, h, acc[j].y);
                    }
                }
#pragma unroll
                for (int e = 1; e < R; ++e) cur[e - 1] = nw[C - e];
            }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");

        // ---- kept outputs: lane writes R consecutive samples ----
        const long m = tile * TO + (long)R * lane;
        float2* o = out + m;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < R; ++j) bad |= !all_finite(acc[j]);
        if (bad) {
            // an inf / NaN sample in the lane's reach: its outputs from the reference's sum
            // (the zero-padded taps would carry it further; fir_exact.hpp)
#pragma unroll 1
            for (int j = 0; j < R; ++j)
                if (m + j < p.n_out) o[j] = fir_exact_output<float2, float>(p, in, hist, m + j);
        } else if (m + R <= p.n_out) {
#pragma unroll
            for (int j = 0; j < R; ++j) o[j] = acc[j];
        } else {
#pragma unroll
            for (int j = 0; j < R; ++j)
                if (m + j < p.n_out) o[j] = acc[j];
        }
    }

    if (blockIdx.x == gridDim.x - 1) {  // stream history carry (see fir_direct.hip)
        float2* hn = static_cast<float2*>(p.hist_next) + ch * (long)(K - 1);
        for (int jj = threadIdx.x; jj < K - 1; jj += kD2Block) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

// ---------------------------------------------------------------------------------
// v3 (D in {2,4,8}): all D phases of one window position are read together.  The D
// samples x[base + D*q + r], r < D, are contiguous: sample r = 0 is phase 0 at window
// position e = q, sample r >= 1 is phase D - r at e = q + 1.  A group of D samples is
// D/2 ds_read_b128 (16 B per lane: 256 B/clk/CU, half the LDS cycles per value of the
// ds_read2_b64 the compiler forms for the per-phase windows of v2).  LDS image: sample s
// at s + 2*floor(s/32) (pairs stay 16-B aligned; lanes 34 samples = 68 dwords apart, so
// every 16-lane group of a b128 read hits 16 distinct 4-bank slots).  R = 32/D outputs
// per lane; a chunk is C = R tap steps (D*R*R packed FMAs per chunk and lane).
constexpr int kD3Front = 48;  // LDS slack (elements) in front of each wave region

template <int D> struct D3Geom {
    static constexpr int R = 32 / D;
    static constexpr int C = R;
};

__host__ __device__ constexpr int d3pad(int s) {
    return s + 2 * (s >= 0 ? s / 32 : -((-s + 31) / 32));
}

struct __attribute__((aligned(8))) f4u { float a, b, c, d; };  // 8-B aligned 16-B access (dwordx4)

template <int D, int NL>
__global__ __launch_bounds__(kD2Block, 2) void fir_direct4_kernel(FirParams p, long ntiles,
                                                                  int wave_lds) {
    constexpr int R = D3Geom<D>::R, C = D3Geom<D>::C, G4 = D / 2;
    static_assert(R == C, "slot schedule assumes R == C");
    extern __shared__ __align__(16) unsigned char smem_raw[];
    using cfloat = const __attribute__((address_space(4))) float;
    typedef float v4f __attribute__((ext_vector_type(4)));

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // kD3Front elements of slack before each wave region: the last chunk's look-ahead
    // reads land there (values unused)
    float2* const wl = reinterpret_cast<float2*>(smem_raw) + kD3Front + wave * wave_lds;

    const long ch = blockIdx.y;
    const float2* __restrict__ in = static_cast<const float2*>(p.in) + ch * p.ld_in;
    const float2* __restrict__ hist = static_cast<const float2*>(p.hist) + ch * (long)(p.K - 1);
    float2* __restrict__ out = static_cast<float2*>(p.out) + ch * p.ld_out;
    cfloat* taps = (cfloat*)(p.taps_pm);
    const int K = p.K;
    const int tpp = p.tpp;
    const int H = D * tpp;
    const int nchunk = tpp / C;
    constexpr long TO = 64L * R;

    float4 st[NL];
    auto tile_s0 = [&](long tile) { return p.i0 + tile * TO * D - H; };
    auto interior = [&](long s0) { return s0 >= 0 && s0 + 128L * NL <= p.n_in; };
    auto load_tile = [&](long tile) {
        const long s0 = tile_s0(tile);
        if (interior(s0)) {
            const f4u* src = reinterpret_cast<const f4u*>(in + s0 + 2 * lane);
#pragma unroll
            for (int i = 0; i < NL; ++i) {
                const f4u v = src[64 * i];
                st[i] = make_float4(v.a, v.b, v.c, v.d);
            }
        }
    };

    long tile = (long)blockIdx.x * (kD2Block / 64) + wave;
    const long tstride = (long)gridDim.x * (kD2Block / 64);
    if (tile < ntiles) load_tile(tile);

    const int wbase = d3pad(H) + 34 * lane;
    const int sbase = 2 * lane + 2 * (lane / 16);

#pragma unroll 1
    for (; tile < ntiles; tile += tstride) {
        {
            const long s0 = tile_s0(tile);
            if (interior(s0)) {
#pragma unroll
                for (int i = 0; i < NL; ++i)
                    *reinterpret_cast<float4*>(wl + sbase + 136 * i) = st[i];
            } else {
#pragma unroll 1
                for (int i = 0; i < NL; ++i) {
                    const long g = s0 + 2 * lane + 128 * i;
                    const float2 a = fetch_c64(in, p.n_in, hist, K, g);
                    const float2 b = fetch_c64(in, p.n_in, hist, K, g + 1);
                    *reinterpret_cast<float4*>(wl + sbase + 136 * i) = make_float4(a.x, a.y, b.x, b.y);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if (tile + tstride < ntiles) load_tile(tile + tstride);

        float2 acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = make_float2(0.f, 0.f);

        const float2* const lb = wl + wbase;
#pragma unroll
        for (int h2 = 0; h2 < G4; ++h2) {
            // this pass: samples r = 2*h2 + u (u = 0, 1) of every group
            auto phase_of = [](int r) { return r == 0 ? 0 : D - r; };
            auto shift_of = [](int r) { return r == 0 ? 0 : 1; };  // X_ph[e] lives in group e - shift
            auto read_half = [&](const float2* lc, int q, float2* g) {
                const v4f v = *reinterpret_cast<const v4f*>(lc + d3pad(D * q) + 2 * h2);
                g[0] = make_float2(v.x, v.y);
                g[1] = make_float2(v.z, v.w);
            };
            float2 HA[C][2], HB[C][2];
            // chunk 0: prev (HB) slot s = group C-1-s, cur (HA) slot s = group -(s+1)
#pragma unroll
            for (int s2 = 0; s2 < C; ++s2) read_half(lb, C - 1 - s2, HB[s2]);
#pragma unroll
            for (int s2 = 0; s2 < C; ++s2) read_half(lb, -(s2 + 1), HA[s2]);

            auto chunk = [&](int c, float2 (&cur)[C][2], float2 (&prev)[C][2]) {
                auto X = [&](int u, int e) -> float2 {
                    const int g = e - shift_of(2 * h2 + u);
                    return g >= 0 ? prev[C - 1 - g][u] : cur[-g - 1][u];
                };
                const float2* ln = lb - 34 * (c + 1);  // next chunk: 32 samples lower
                // this chunk's C taps of the pass's two phases: contiguous, wave-uniform
                cfloat* tq0 = taps + (unsigned)(phase_of(2 * h2) * tpp + c * C);
                cfloat* tq1 = taps + (unsigned)(phase_of(2 * h2 + 1) * tpp + c * C);
                float hv[2][C];
#pragma unroll
                for (int a = 0; a < C; ++a) {
                    hv[0][a] = tq0[a];
                    hv[1][a] = tq1[a];
                }
#pragma unroll
                for (int a = 0; a < C; ++a) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const float h = hv[u][a];
#pragma unroll
                        for (int j = 0; j < R; ++j) {
                            const float2 x = X(u, j - a);
                            acc[j].x = fmaf(x.x, h, acc[j].x);
                            acc[j].y = fmaf(x.y, h, acc[j].y);
                        }
                    }
                    // prev slot a is free from here on; the fences keep the refill from
                    // being hoisted above the FMAs that still read the old contents
                    __builtin_amdgcn_sched_barrier(0);
                    read_half(ln, -(a + 1), prev[a]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            int c = 0;
#pragma unroll 1
            for (; c + 1 < nchunk; c += 2) {
                chunk(c, HA, HB);
                chunk(c + 1, HB, HA);
            }
            if (c < nchunk) chunk(c, HA, HB);
        }

        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");

        const long m = tile * TO + (long)R * lane;
        float2* o = out + m;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < R; ++j) bad |= !all_finite(acc[j]);
        if (bad) {
            // an inf / NaN sample in the lane's reach: its outputs from the reference's sum
            // (the zero-padded taps would carry it further; fir_exact.hpp)
#pragma unroll 1
            for (int j = 0; j < R; ++j)
                if (m + j < p.n_out) o[j] = fir_exact_output<float2, float>(p, in, hist, m + j);
        } else if (m + R <= p.n_out) {
#pragma unroll
            for (int j = 0; j < R; j += 2)
                *reinterpret_cast<f4u*>(o + j) = f4u{acc[j].x, acc[j].y, acc[j + 1].x, acc[j + 1].y};
        } else {
#pragma unroll
            for (int j = 0; j < R; ++j)
                if (m + j < p.n_out) o[j] = acc[j];
        }
    }

    if (blockIdx.x == gridDim.x - 1) {
        float2* hn = static_cast<float2*>(p.hist_next) + ch * (long)(K - 1);
        for (int jj = threadIdx.x; jj < K - 1; jj += kD2Block) {
            const long g = p.n_in - (long)(K - 1) + jj;
            hn[jj] = g >= 0 ? in[g] : hist[g + (K - 1)];
        }
    }
}

inline int cu_count() {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t prop;
        n_cu = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    }
    return n_cu;
}

template <int D, int NL>
int launch_d3(const FirParams& p, hipStream_t s) {
    const int wave_lds = d3pad(128 * NL) + 2;  // elements (even -> 16-B multiple)
    const size_t lds = ((size_t)wave_lds * (kD2Block / 64) + kD3Front) * sizeof(float2);
    const long ntiles = ceil_div(p.n_out, 64L * D3Geom<D>::R);
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
    const long want = ceil_div(ntiles, kD2Block / 64);
    long cap = ((long)cu_count() * per_cu + p.nch - 1) / p.nch;
    if (cap < 1) cap = 1;
    const long gx = std::max(1L, std::min(want, cap));
    dim3 grid((unsigned)gx, (unsigned)p.nch);
    hipLaunchKernelGGL((fir_direct4_kernel<D, NL>), grid, dim3(kD2Block), lds, s, p, ntiles,
                       wave_lds);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

template <int D>
int dispatch_d3(const FirParams& p, hipStream_t s) {
    const int H = D * p.tpp;
    const int nl = (H + 2048 + 127) / 128;  // b128 loads per lane
    if (nl <= 17) return launch_d3<D, 17>(p, s);
    if (nl <= 18) return launch_d3<D, 18>(p, s);
    if (nl <= 20) return launch_d3<D, 20>(p, s);
    if (nl <= 24) return launch_d3<D, 24>(p, s);
    return SDRGPU_ERR_UNSUPPORTED;
}

template <int D, int NL>
int launch_d2(const FirParams& p, hipStream_t s) {
    using G = D2Geom<D>;
    // wave region holds all 64*NL staged samples (>= H + 64*SPAN), padded
    const int wave_lds = (d2pad<G::SPAN>(64 * NL) + 2) & ~1;  // elements, 16-B multiple
    const size_t lds = (size_t)wave_lds * sizeof(float2) * (kD2Block / 64);
    const long ntiles = ceil_div(p.n_out, 64L * G::R);
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t prop;
        n_cu = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    }
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
    long want = ceil_div(ntiles, kD2Block / 64);
    long cap = ((long)n_cu * per_cu + p.nch - 1) / p.nch;
    if (cap < 1) cap = 1;
    const long gx = std::max(1L, std::min(want, cap));
    dim3 grid((unsigned)gx, (unsigned)p.nch);
    hipLaunchKernelGGL((fir_direct2_kernel<D, NL>), grid, dim3(kD2Block), lds, s, p, ntiles,
                       wave_lds);
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

template <int D>
int dispatch_d2(const FirParams& p, hipStream_t s) {
    constexpr int SPAN = D2Geom<D>::SPAN;
    const int H = D * p.tpp;
    const int nl = SPAN + (H + 63) / 64;  // loads per lane
    if (nl <= SPAN + 2) return launch_d2<D, SPAN + 2>(p, s);
    if (nl <= SPAN + 4) return launch_d2<D, SPAN + 4>(p, s);
    if (nl <= SPAN + 8) return launch_d2<D, SPAN + 8>(p, s);
    if (nl <= SPAN + 16) return launch_d2<D, SPAN + 16>(p, s);
    return SDRGPU_ERR_UNSUPPORTED;
}

}  // namespace

bool fir_direct2_supported(const FirParams& p) {
    if (p.sample_kind != SDRGPU_C64 || p.tap_kind != SDRGPU_F32) return false;
    if (!(p.D == 1 || p.D == 2 || p.D == 4 || p.D == 8)) return false;
    if (p.tpp % kD2Chunk) return false;
    return (long)p.D * p.tpp <= 1024;
}

int fir_direct2_launch(const FirParams& p, hipStream_t s) {
    if (!fir_direct2_supported(p)) return SDRGPU_ERR_UNSUPPORTED;
    switch (p.D) {
    case 1: return dispatch_d2<1>(p, s);
    case 2: return dispatch_d3<2>(p, s);
    case 4: return dispatch_d3<4>(p, s);
    case 8: return dispatch_d3<8>(p, s);
    default: return SDRGPU_ERR_UNSUPPORTED;
    }
}

}  // namespace sdrgpu
