// fir_mxi.hip -- rtl_tcp u8 I/Q FIR (decimate by 4, or no decimation) on the int8 MFMAs
// (gfx950): the fused ingest of SURVEY 8f-1 with exact integer products.
//
// Semantics: RtlTcpSignal::next (reference src/rtltcp.rs:156-164: x = (v - 128) / 128) feeding
// Fir::apply + Decimate (src/filter/fir.rs:23-32, src/filter/convolve.rs:13-15,
// src/signal/adapters/mod.rs:30-37) with real taps: y[m] = sum_k h[k] x[i0 + 4m - k], zero
// history before the stream start.
//
// Why int8: a u8 code minus 128 is an exact int8 (the XOR with 0x80 of the byte), so the
// samples need no conversion and no split at all.  The taps go in as integers too:
// t = rint(h 2^S) with |t| <= 2^22 (S = tap_scale_exp + 7), written as three balanced int8
// digits t = 2^16 d2 + 2^8 d1 + d0.  v_mfma_i32_16x16x64_i8 then sums digit x sample
// products exactly in i32 (|sum| <= 5 x 64 x 128^2 < 2^23 per digit), and the tile's outputs
// are (2^16 C2 + 2^8 C1 + C0) 2^-(S+7) with two f32 roundings -- the one approximation is the
// taps' rounding to integers, <= 2^-22 of max |h| (the fp16 kernel's hh + hl: about the same).
//
// Against the fp16 form of the same tiles (fir_mxh.hip, U8 = true): K = 64 per MFMA at the
// same 16 cycles, so 3 digits x 5 chunks x 2 components = 30 MFMAs per 256-output tile
// instead of 40; one byte per sample in LDS, so a chunk's B fragment is one ds_read_b128 per
// component (10 per tile instead of 20) and a window buffer is 2 x 1280 B; staging is a
// byte permute (v_perm_b32 splits I from Q) instead of four converts per sample pair.
//
// Tiles and GEMM shape: a tile is 256 kept outputs = 1024 new samples; C[16 x 16] with rows
// u = output offset in a 16-output block (A = taps: A[u][p] = h[4u + 3 - delta + H - p], in
// registers) and columns v = the tile's 16 blocks (B = samples: B[p][v] = window[64 v + p]);
// K = 320 window samples = 5 chunks of 64 (H = 256 history samples).
//
// D = 8: tiles of 2048 new samples (one column set), K = 6 chunks (K + 127 <= 384; 4 for
// K <= 129), the 16-byte units XOR-swizzled within 256-byte lines (win_addr<8>).
// D = 1 (the same stream without Decimate) and D = 2: rows are 16 outputs D samples apart,
// columns blocks 16 D samples apart, K = 5 chunks cover K + 15 D + D - 1 <= 320; a tile is
// 4 / D 256-output column sets over one staged window of H + 1024 samples (so the raw-tile
// pipeline is the D = 4 one), and the LDS layout is linear (conflict free for those spacings).
//
// LDS (wave-private, no barriers): two window buffers (compute tile k from one while tile
// k + 1 is staged into the other), each two planes (I, Q) of H + 1024 int8 samples in rows of
// 64 B; window sample b sits at 64 (b >> 6) + 16 (((b >> 4) & 3) ^ ((b >> 7) & 3)) + (b & 15).
// A chunk-c fragment read (lane v + 16 g reads row v + c, 16-B unit g) is bank-conflict free
// in every 16-lane group of a ds_read_b128 for every c, and the staging writes of 8 samples
// per lane (ds_write_b64, 32 lanes = 4 whole rows) are too.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "fir_mxi.hpp"

namespace sdrgpu {

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;  // two waves per SIMD (one workgroup per CU)
constexpr int kBlock = 64 * kWaves;
constexpr int kCs = 1;        // D = 4: 256-output column sets per staged window (tile)
constexpr int kCs1 = 4;       // D = 1: four sets, so a tile is 1024 new samples as at D = 4
constexpr int kCs2 = 2;       // D = 2: two sets
constexpr int kRunTiles = 8;  // per-workgroup runs of 8 x 256 outputs (as the fp16 u8 launch)

// (2^16 C2 + 2^8 C1 + C0) 2^-(S+7) as fmaf(C2, sc2, fmaf(C1, sc1, C0 sc0)), written as VOP3
// v_mul_f32 / v_fma_f32: plain C++ lets the compiler pair the re and im combinations into
// packed-f32 ops, and packed-f32 results went wrong beside another wave's MFMAs on the SIMD in
// this library twice (profiles/r06_pkfault.txt) -- this kernel runs two waves
// per SIMD.  Same roundings, same bytes.
__device__ __forceinline__ float digits_f32(int c0, int c1, int c2, float sc0, float sc1, float sc2) {
    const float a = (float)c0, b = (float)c1, d = (float)c2;
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(sc0));
    asm("v_fma_f32 %0, %1, %2, %0" : "+v"(r) : "v"(b), "v"(sc1));
    asm("v_fma_f32 %0, %1, %2, %0" : "+v"(r) : "v"(d), "v"(sc2));
    return r;
}

template <int NC, int CS, int D>
struct GeoI {
    static constexpr int HR = 64 * NC - 16 * D;   // history samples a tile's window needs
    static constexpr int H = (HR + 63) / 64 * 64; // staged history (whole 64-sample rows)
    static constexpr int OFF = H - HR;            // window offset inside the buffer
    static constexpr int TI = 256 * D * CS;       // new samples per tile
    static constexpr int NG = TI / 512;           // raw groups of 512 samples per tile
    static constexpr int WL = H + TI;             // window samples = bytes per plane
    static constexpr int WINB = 2 * WL;           // bytes per window buffer (I, Q planes)
    static constexpr int WAVE = 2 * WINB;         // bytes per wave (two buffers)
    static constexpr int HL = 64 - H / 8;         // first lane holding history (8 samples/lane)
    static_assert(TI % 512 == 0 && H <= 512 && CS * NC >= 2, "geometry");
    static_assert(D != 4 || OFF == 0, "geometry");
};

struct MxiParams {
    const unsigned char* in;  // interleaved u8 I/Q
    long ld_in, n_in;         // per channel, in samples (2 bytes)
    const float2* hist;
    float2* hist_next;
    const unsigned char* dummy;  // >= 2 TI bytes readable (one raw tile): target of clamped prefetches
    long n_out;
    int K;
    int delta;  // D - 1 - i0
    int S;      // taps scaled by 2^S before the digit split
    const float* taps;
    float2* out;
    long ld_out;
    long tpc, spc, seg_tiles, units;
    int vec_out;
};

__device__ __forceinline__ i32x4 mfma8(const i32x4& a, const u32x4& b, i32x4 c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, __builtin_bit_cast(i32x4, b), c, 0, 0, 0);
}

// back to the u8 code of an exactly-converted sample (history written by this handle)
__device__ __forceinline__ unsigned iq_u8(float2 v) {
    return (unsigned)(v.x * 128.0f + 128.0f) | ((unsigned)(v.y * 128.0f + 128.0f) << 8);
}
__device__ __forceinline__ float2 u8_iq(unsigned short w) {
    return make_float2(((float)(w & 0xffu) - 128.0f) / 128.0f, ((float)(w >> 8) - 128.0f) / 128.0f);
}
// 8 samples (j .. j + 7) as 16 raw bytes, with history / zero (code 128) fill: stream start/end
__device__ __forceinline__ u32x4 fetch8(const unsigned short* in, const float2* hist, long j,
                                     long n_in, int K) {
    u32x4 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        unsigned w = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const long i = j + 2 * q + e;
            const bool inb = (i >= 0) & (i < n_in);
            const bool inh = (i < 0) & (i >= -(long)(K - 1));
            const unsigned a = in[inb ? i : 0];
            const unsigned b = iq_u8(hist[inh ? i + (K - 1) : 0]);
            w |= (inb ? a : (inh ? b : 0x8080u)) << (16 * e);
        }
        r[q] = w;
    }
    return r;
}

// window sample b -> byte offset inside a plane: D = 4 swizzles 16-byte units within 64-byte
// rows; D = 8 (blocks 128 samples apart) XORs the 16-byte unit within its 256-byte line with
// 2 (line & 3); at D = 1 and 2 (blocks 16 / 32 samples apart) the linear layout is already
// conflict free
template <int D>
__device__ __forceinline__ int win_addr(int b) {
    if constexpr (D == 1 || D == 2) return b;
    if constexpr (D == 8) return (b & ~255) | ((((b >> 4) & 15) ^ (2 * ((b >> 8) & 3))) << 4) | (b & 15);
    return 64 * (b >> 6) + 16 * (((b >> 4) & 3) ^ ((b >> 7) & 3)) + (b & 15);
}

// 8 raw I/Q pairs -> 8 int8 I at plane 0, 8 int8 Q at plane 1 (byte a of the buffer)
template <int WL>
__device__ __forceinline__ void put8(char* lds, int a, const u32x4& w) {
    const unsigned w0 = w[0] ^ 0x80808080u, w1 = w[1] ^ 0x80808080u;
    const unsigned w2 = w[2] ^ 0x80808080u, w3 = w[3] ^ 0x80808080u;
    uint2 re, im;
    re.x = __builtin_amdgcn_perm(w1, w0, 0x06040200u);
    re.y = __builtin_amdgcn_perm(w3, w2, 0x06040200u);
    im.x = __builtin_amdgcn_perm(w1, w0, 0x07050301u);
    im.y = __builtin_amdgcn_perm(w3, w2, 0x07050301u);
    *reinterpret_cast<uint2*>(lds + a) = re;
    *reinterpret_cast<uint2*>(lds + a + WL) = im;
}

template <int NC, int CS, int D>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2, 2)))
void fir_mxi_kernel(MxiParams p) {
    using G = GeoI<NC, CS, D>;
    constexpr int H = G::H, HR = G::HR, WL = G::WL, WINB = G::WINB, HL = G::HL;
    constexpr int TI = G::TI, NG = G::NG;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    claim_simd_half();  // two waves fill the SIMD: nothing else shares it (common.hpp)
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv >= kWaves / 2) __builtin_amdgcn_s_setprio(1);
    const int g = lane >> 4, v = lane & 15;
    const int K = p.K;
    const int base = wv * G::WAVE;

    // ---- A: tap Toeplitz fragments as three balanced int8 digits ----
    i32x4 ad[NC][3];
    {
        const float tsc = __builtin_amdgcn_ldexpf(1.0f, p.S);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                unsigned d0w = 0, d1w = 0, d2w = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int pidx = 64 * c + 16 * g + 4 * q + e;
                    const int k = D * v + D - 1 - p.delta + HR - pidx;
                    const bool ok = (k >= 0) & (k < K);
                    const float hk = p.taps[ok ? k : 0];
                    const int t = ok ? (int)rintf(hk * tsc) : 0;
                    const int d0 = ((t + 128) & 255) - 128;
                    const int t1 = (t - d0) >> 8;
                    const int d1 = ((t1 + 128) & 255) - 128;
                    const int d2 = (t1 - d1) >> 8;
                    d0w |= (unsigned)(d0 & 255) << (8 * e);
                    d1w |= (unsigned)(d1 & 255) << (8 * e);
                    d2w |= (unsigned)(d2 & 255) << (8 * e);
                }
                ad[c][0][q] = (int)d0w;
                ad[c][1][q] = (int)d1w;
                ad[c][2][q] = (int)d2w;
            }
        }
    }
    int rb[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if constexpr (D == 4) {
            const int r = v + c;
            rb[c] = base + 64 * r + 16 * (g ^ ((r >> 1) & 3));
        } else if constexpr (D == 8) {
            rb[c] = base + win_addr<8>(G::OFF + 128 * v + 64 * c + 16 * g);
        } else {
            rb[c] = base + G::OFF + 16 * D * v + 64 * c + 16 * g;
        }
    }
    // staging addresses: lane l stages new samples 8 l + 512 k (k < NG; at D = 1, 2 and 4 the
    // swizzle is the same for every k, so group k sits 512 k bytes on, but not at D = 8) and,
    // if l >= HL, history samples 8 (l - HL)
    const int wa0 = base + win_addr<D>(H + 8 * lane);
    auto wa = [&](int k) __attribute__((always_inline)) {
        if constexpr (D == 8) return base + win_addr<8>(H + 512 * k + 8 * lane);
        return wa0 + 512 * k;
    };
    const int wh = base + win_addr<D>(8 * (lane >= HL ? lane - HL : 0));

    // ---- the wave's tile stream (fir_mxh.hip's cursors, per-workgroup blocked units) ----
    struct Cur {
        long u, t, ch, tu, nt;
        bool ok;
    };
    const long ub1 = ((long)blockIdx.x + 1) * p.units / gridDim.x;
    auto seek = [&](Cur& c, long u) __attribute__((always_inline)) {
        c.u = u;
        c.t = 0;
        c.ok = u < ub1;
        c.ch = c.ok ? u / p.spc : 0;
        c.tu = (u - c.ch * p.spc) * p.seg_tiles;
        c.nt = c.ok ? std::min(p.seg_tiles, p.tpc - c.tu) : 0;
        if (c.ok && c.nt <= 0) c.ok = false;
    };
    auto adv = [&](Cur& c) __attribute__((always_inline)) {
        if (!c.ok) return;
        if (++c.t >= c.nt) seek(c, c.u + kWaves);
    };
    const long n_in = p.n_in;
    auto tile_j0 = [&](const Cur& c) { return (long)TI * (c.tu + c.t); };
    auto tile_fast = [&](const Cur& c) { return (long)TI * (c.tu + c.t + 1) <= n_in; };
    auto chan = [&](const Cur& c) { return p.in + 2 * c.ch * p.ld_in; };
    auto load_tile = [&](u32x4 (&dst)[NG], const Cur& c) __attribute__((always_inline)) {
        const long j0 = tile_j0(c);
        if (tile_fast(c)) {
            const u32x4* q = reinterpret_cast<const u32x4*>(chan(c) + 2 * j0);
#pragma unroll
            for (int k = 0; k < NG; ++k) dst[k] = __builtin_nontemporal_load(q + 64 * k + lane);
        } else {
            asm volatile("" ::: "memory");
            const unsigned short* in = reinterpret_cast<const unsigned short*>(chan(c));
            const float2* hist = p.hist + c.ch * (long)(K - 1);
#pragma unroll
            for (int k = 0; k < NG; ++k) dst[k] = fetch8(in, hist, j0 + 512 * k + 8 * lane, n_in, K);
        }
    };
    // the H samples before tile c, 8 per lane in lanes HL..63 (the tail layout of a raw tile)
    auto load_hist = [&](u32x4& dst, const Cur& c) __attribute__((always_inline)) {
        const long j = tile_j0(c) - H + 8 * (lane >= HL ? lane - HL : 0);
        if (tile_j0(c) >= H && tile_j0(c) <= n_in) {
            dst = *reinterpret_cast<const u32x4*>(chan(c) + 2 * j);
        } else {
            asm volatile("" ::: "memory");
            dst = fetch8(reinterpret_cast<const unsigned short*>(chan(c)),
                         p.hist + c.ch * (long)(K - 1), j, n_in, K);
        }
    };

    Cur cm, st, ld;
    seek(cm, (long)blockIdx.x * p.units / gridDim.x + wv);
    if (cm.ok) {
        u32x4 nx[NG], hr;
        load_hist(hr, cm);
        load_tile(nx, cm);
        if (lane >= HL) put8<WL>(smem, wh, hr);
#pragma unroll
        for (int k = 0; k < NG; ++k) put8<WL>(smem, wa(k), nx[k]);
        st = cm;
        adv(st);
        if (st.ok && st.t == 0) load_hist(hr, st);
        else hr = nx[NG - 1];
        if (st.ok) load_tile(nx, st);
        ld = st;
        adv(ld);

        const float sc0 = __builtin_amdgcn_ldexpf(1.0f, -(p.S + 7));
        const float sc1 = sc0 * 256.0f, sc2 = sc0 * 65536.0f;
        auto body = [&](auto tau_c) __attribute__((always_inline)) {
            constexpr int TAU = decltype(tau_c)::value;
            constexpr int WN = (1 - TAU) * WINB;  // staging buffer offset
            const bool fast2 = ld.ok && tile_fast(ld);
            const bool ld_run = ld.ok && ld.t == 0;  // tile k+2 opens a run: reload history
            const u32x4* src2 = reinterpret_cast<const u32x4*>(
                fast2 ? chan(ld) + 2 * tile_j0(ld) : p.dummy);
            i32x4 acc[2][3];
            u32x4 fb[2][2];
            // column set j reads 256 D samples further into the window (D = 4: 16 rows, the
            // same swizzle)
            auto read_frags = [&](u32x4 (&f)[2], int i) __attribute__((always_inline)) {
                const int a = rb[i % NC] + TAU * WINB + 256 * D * (i / NC);
                f[0] = *reinterpret_cast<const u32x4*>(smem + a);
                f[1] = *reinterpret_cast<const u32x4*>(smem + a + WL);
            };
            read_frags(fb[0], 0);
            const u32x4 keep = nx[NG - 1];
            float2* __restrict__ out = p.out + cm.ch * p.ld_out;
#pragma unroll
            for (int i = 0; i < CS * NC; ++i) {
                const int j = i / NC, c = i % NC;
                if (c == 0) {
#pragma unroll
                    for (int d = 0; d < 3; ++d) acc[0][d] = acc[1][d] = i32x4{0, 0, 0, 0};
                }
                if (i + 1 < CS * NC) read_frags(fb[(i + 1) & 1], i + 1);
                __builtin_amdgcn_sched_barrier(0);
                const u32x4(&f)[2] = fb[i & 1];
#pragma unroll
                for (int d = 2; d >= 0; --d) {
                    acc[0][d] = mfma8(ad[c][d], f[0], acc[0][d]);
                    acc[1][d] = mfma8(ad[c][d], f[1], acc[1][d]);
                }
                if (i == 0) {  // window k+1's history; then tile k+2's, if it opens a run
                    if (lane >= HL) put8<WL>(smem, WN + wh, hr);
                    if (ld_run) load_hist(hr, ld);
                }
#pragma unroll
                for (int k = 0; k < NG; ++k) {  // group k at iteration k + 1 (the last takes the rest)
                    if ((k + 1 < CS * NC ? k + 1 : CS * NC - 1) != i) continue;
                    put8<WL>(smem, WN + wa(k), nx[k]);
                    nx[k] = __builtin_nontemporal_load(src2 + 64 * k + lane);
                }
                if (c == NC - 1) {  // column set j complete: scale and store its 256 outputs
                    const long m0 = (cm.tu + cm.t) * (256L * CS) + 256 * j;
                    const long m = m0 + 16 * v + 4 * g;
                    float yr[4], yi[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        yr[q] = digits_f32(acc[0][0][q], acc[0][1][q], acc[0][2][q], sc0, sc1, sc2);
                        yi[q] = digits_f32(acc[1][0][q], acc[1][1][q], acc[1][2][q], sc0, sc1, sc2);
                    }
                    if (p.vec_out && m0 + 256 <= p.n_out) {
                        // line-complete stores (fir_mxh.hip): lanes v and v^1 swap one 16-B half
                        const bool ev = (v & 1) == 0;
                        const f32x4 y0 = {yr[0], yi[0], yr[1], yi[1]};
                        const f32x4 y1 = {yr[2], yi[2], yr[3], yi[3]};
                        f32x4 rx;
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            rx[q] = __int_as_float(__builtin_amdgcn_mov_dpp(
                                __float_as_int(ev ? y1[q] : y0[q]), 0xB1, 0xf, 0xf, false));
                        const long mp = m0 + 16 * (v ^ 1) + 4 * g;
                        f32x4* o4 = reinterpret_cast<f32x4*>(out + (ev ? m : mp + 2));
                        f32x4* p4 = reinterpret_cast<f32x4*>(out + (ev ? mp : m + 2));
                        __builtin_nontemporal_store(ev ? y0 : rx, o4);
                        __builtin_nontemporal_store(ev ? rx : y1, p4);
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (m + q < p.n_out) out[m + q] = make_float2(yr[q], yi[q]);
                    }
                }
            }
            if (!ld_run) hr = keep;  // tile k+2 continues the run: its history is k+1's tail
            if (!fast2 && ld.ok) load_tile(nx, ld);
            cm = st;
            st = ld;
            adv(ld);
        };
        while (cm.ok) {
            body(std::integral_constant<int, 0>());
            if (!cm.ok) break;
            body(std::integral_constant<int, 1>());
        }
    }

    if (p.hist_next) {  // stream history carry, spread over the whole grid
        const long nch = p.units / p.spc;
        for (long j = (long)blockIdx.x * kBlock + threadIdx.x; j < nch * (K - 1);
             j += (long)gridDim.x * kBlock) {
            const long ch = j / (K - 1), jj = j - ch * (K - 1);
            const float2* hic = p.hist + ch * (long)(K - 1);
            const long gidx = p.n_in - (long)(K - 1) + jj;
            const unsigned short* inb = reinterpret_cast<const unsigned short*>(p.in) + ch * p.ld_in;
            p.hist_next[j] = gidx >= 0 ? u8_iq(inb[gidx]) : hic[gidx + (K - 1)];
        }
    }
}

int mxi_nc(int K, int D) {
    const int need = (K + 16 * D - 1 + 63) / 64;  // 64 NC >= K + 15 D + D - 1
    if (D == 8) return need <= 4 ? 4 : (need <= 6 ? 6 : 0);
    return need <= 3 ? 3 : (need <= 5 ? 5 : 0);
}

}  // namespace

int fir_mxi_supported(const FirParams& fp, int tap_scale_exp) {
    if (fp.sample_kind != SDRGPU_CU8 || fp.tap_kind != SDRGPU_F32) return 0;
    if (!(fp.D == 8 || fp.D == 4 || fp.D == 2 || fp.D == 1) || fp.K < 1 || fp.K > 257) return 0;
    if (mxi_nc(fp.K, fp.D) == 0 || fp.i0 < 0 || fp.i0 >= fp.D) return 0;
    // taps as 23-bit integers: 2^S and the output scale 2^-(S + 7) stay normal floats
    if (tap_scale_exp + 14 > 126 || tap_scale_exp + 7 < -126) return 0;
    // 16-byte loads of 8 samples: channel bases stay 16-byte aligned
    if ((reinterpret_cast<uintptr_t>(fp.in) & 15) != 0 || (fp.nch > 1 && (fp.ld_in & 7)))
        return 0;
    return 1;
}

int fir_mxi_launch(const FirParams& fp, const float* d_taps, int tap_scale_exp,
                   const void* d_dummy, int cus, hipStream_t s) {
    if (!fir_mxi_supported(fp, tap_scale_exp) || !d_dummy) return SDRGPU_ERR_UNSUPPORTED;
    const int D = fp.D;
    // a clamped prefetch reads one whole raw tile (NG groups x 64 lanes x 16 B = 2 TI bytes)
    // from the dummy buffer: 4 KiB at D = 8
    const long tile_bytes = 2L * 256 * D * (D >= 4 ? kCs : (D == 2 ? kCs2 : kCs1));
    if ((long)fir_mxh_dummy_bytes() < tile_bytes) return SDRGPU_ERR_UNSUPPORTED;
    const int NC = mxi_nc(fp.K, D);
    MxiParams p;
    p.in = static_cast<const unsigned char*>(fp.in);
    p.ld_in = fp.ld_in;
    p.n_in = fp.n_in;
    p.hist = static_cast<const float2*>(fp.hist);
    p.hist_next = fp.K > 1 ? static_cast<float2*>(fp.hist_next) : nullptr;
    p.dummy = static_cast<const unsigned char*>(d_dummy);
    p.n_out = fp.n_out;
    p.K = fp.K;
    p.delta = (int)(D - 1 - fp.i0);
    p.S = tap_scale_exp + 7;
    p.taps = d_taps;
    p.out = static_cast<float2*>(fp.out);
    p.ld_out = fp.ld_out;
    p.vec_out = ((reinterpret_cast<uintptr_t>(fp.out) & 15) == 0 &&
                 (fp.nch == 1 || !(fp.ld_out & 1)))
                    ? 1
                    : 0;
    const long nch = fp.nch;
    const int cs = D >= 4 ? kCs : (D == 2 ? kCs2 : kCs1);
    p.tpc = ceil_div(std::max(0L, fp.n_out), 256L * cs);
    p.seg_tiles = std::max(1L, std::min<long>(std::max(1, kRunTiles / cs), p.tpc));
    p.spc = std::max(1L, ceil_div(p.tpc, p.seg_tiles));
    p.units = nch * p.spc;
    const long blocks = std::max(1L, std::min((long)cus, ceil_div(p.units, kWaves)));
#define SDRGPU_MXI_GO(NCC, CSS, DD)                                                            \
    hipLaunchKernelGGL((fir_mxi_kernel<NCC, CSS, DD>), dim3(blocks), dim3(kBlock),             \
                       (size_t)kWaves * (GeoI<NCC, CSS, DD>::WAVE), s, p)
    if (D == 8 && NC == 6) SDRGPU_MXI_GO(6, kCs, 8);
    else if (D == 8) SDRGPU_MXI_GO(4, kCs, 8);
    else if (D == 4 && NC == 5) SDRGPU_MXI_GO(5, kCs, 4);
    else if (D == 4) SDRGPU_MXI_GO(3, kCs, 4);
    else if (D == 2 && NC == 5) SDRGPU_MXI_GO(5, kCs2, 2);
    else if (D == 2) SDRGPU_MXI_GO(3, kCs2, 2);
    else if (NC == 5) SDRGPU_MXI_GO(5, kCs1, 1);
    else SDRGPU_MXI_GO(3, kCs1, 1);
#undef SDRGPU_MXI_GO
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

}  // namespace sdrgpu
