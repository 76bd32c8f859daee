// fir_mxh.hip -- LDS-staged MFMA direct-form FIR, decimate by 4, on a per-tile scaled
// two-way fp16 split (gfx950): two waves per SIMD.
//
// Semantics: Fir::apply + Decimate (reference src/filter/fir.rs:23-32,
// src/filter/convolve.rs:13-15, src/signal/adapters/mod.rs:30-37) for complex samples and
// real taps: y[m] = sum_k h[k] x[i0 + 4m - k], zero history before the stream start.
//
// Same GEMM shape, tiles and conflict-free LDS swizzle as the exact bf16x3 variant kept in
// tools/experiments/fir_mxl.hip (read that header first); what changes is the operand format, which halves both the MFMA work and the
// LDS footprint so that two waves share each SIMD (one's VALU/LDS staging and memory waits
// overlap the other's MFMAs):
//   * every tile's window (1024 new samples + H history samples) is staged with its own
//     power-of-two scale 2^s, s = 15 - exponent(max |x| over the window), so the scaled
//     samples lie below 2^15 and fit fp16; each scaled sample is split into
//     xh = rtz_f16(x) and xl = rtz_f16(x - xh) (x is represented to < 2^-20 relative);
//   * taps likewise: h 2^sh = hh + hl (round-to-nearest, host-chosen sh);
//   * x h ~= xh hh + xh hl + xl hh on v_mfma_f32_16x16x32_f16 (3 MFMAs per component
//     instead of the bf16 path's 6; the dropped xl hl < 2^-20 |x h|), and the tile's
//     outputs are rescaled by 2^-(s + sh) before the store.
// The scale is per tile, so a sample's relative precision is 2^-20 of the largest sample
// within the same ~1280-sample window (the reference's own f32 sum has a rounding error of
// 2^-24 of its largest term); samples more than 2^-24 below that maximum (or |x| < 2^-111)
// fall into fp16 subnormals.  f32's exponent range is otherwise kept (any input scale).
//
// LDS per wave: a ring of R = H + 2 TI samples in 4 planes (hi/lo x re/im, 2 B each).  Even
// tiles of the wave's stream use window [0, H + TI), odd tiles [TI, R): an odd tile's history
// (the H samples before it) is the tail of the even tile's window, already staged -- when the
// odd tile continues the even tile's run and keeps its scale (sticky scale below), it is not
// staged again.  Tile t computes from its window while tile t+1 is staged into the other; the
// even window's last H samples overlap the odd window's history, so an even tile's last NH
// groups (and an odd tile's history, when it has to be staged) are written after the MFMA
// loop of the tile being computed.  4 x 2304 x 2 B = 18 KiB at NCH = 10 (was 20 KiB with
// two separate window buffers).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "fir_kernels.hpp"

namespace sdrgpu {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;               // two waves per SIMD
constexpr int kBlock = 64 * kWaves;
// D = 1 tiles: four 256-output column sets share one staged window (one set: 2.62 ms at
// configs[4], three: 2.48, profiles/r02_fir_d1_cs.txt; four fit only in the LDS ring: 2.037
// vs 2.079 ms for three in the driver window, profiles/r05_fir_ring_ab.txt); 8 groups keep
// one raw tile in flight
constexpr int kCs1 = 4;
// D = 2 tiles: two 256-output column sets over one 1024-sample window (the D = 4 raw pipeline)
constexpr int kCs2 = 2;
// D = 4 runs.  c64 samples: runs of 2 tiles dealt grid-strided, so at any moment the whole
// chip streams one contiguous window (2048 waves x 16 KiB): 0.441 ms, against 0.460 for the
// same runs in per-workgroup ranges, 0.486-0.488 for per-workgroup runs of 8 (round 3 s3), and
// 0.478 / 0.486-0.491 / 0.528 for grid-strided runs of 4 / 8 / 1 (steady-state A/B,
// profiles/r03s4_run_length_ab.txt).  u8 ingest: per-workgroup runs of 8 (every variant
// within noise there).
constexpr int kRunTiles = 2;
constexpr int kRunTilesU8 = 8;
// Staging schedule: the next window's groups are split and written kStagePerChunk per MFMA chunk
// (groups 0-3 after chunk 0, 4-7 after chunk 1), so the raw-tile loads that reuse their
// registers are issued early in the body and have most of it to land.  Round 6, alternating
// same-box A/Bs (profiles/r06_stage_burst_ab.txt), outputs bit-identical to one group per chunk:
// configs[1] steady state 0.4400 -> 0.4289 ms (2 per chunk 0.4323, 8 0.4346), driver window
// 0.501 -> 0.504 ms (noise); configs[4] bank 1.967 -> 1.954 ms in the window.
constexpr int kStagePerChunk = 4;
// wave_scale of a window holding inf or NaN (exact_tile below): exp2i of it is inf (that window's
// staged values are never used), and the sticky-scale test neither keeps it into a finite window
// nor keeps a finite scale into it
constexpr int kNonFinite = 1 << 16;

// CS: 256-output MFMA column sets per tile.  D = 1 stages the window's history once for CS
// column sets (the history is 1.5x a 256-sample set, so re-staging it per set dominated)
template <int NCH, int D = 4, int CS = 1>
struct GeoH {
    static constexpr int TO = 256 * CS;            // outputs per tile
    static constexpr int TI = TO * D;              // new samples per tile
    static constexpr int HR = 32 * NCH - 16 * D;   // history samples a tile's windows need
    static constexpr int H = (HR + 127) / 128 * 128;  // staged history (128-sample groups)
    static constexpr int OFF = H - HR;             // window offset inside the buffer
    static constexpr int R = H + 2 * TI;           // ring samples per plane
    static constexpr int PLB = 2 * R;              // bytes per plane
    static constexpr int WODD = 2 * TI;            // byte offset of the odd tiles' window
    static constexpr int WAVE = 4 * PLB;           // bytes per wave
    static constexpr int NG = TI / 128;            // 128-sample groups per tile
    static constexpr int NH = H / 128;             // history groups
    static_assert(HR > 0 && (D == 1 || ((D == 4 || D == 2) && OFF == 0)), "geometry");
    // even history [0, H) must stay clear of the odd window [TI, R); the row swizzles of D = 4
    // (period 16 rows of 64 samples) and D = 2 (8 rows of 32) repeat every TI samples
    static_assert(TI >= H && (D == 1 || TI % 1024 == 0), "ring");
    static_assert(kWaves * WAVE <= 160 * 1024, "LDS");
};

struct MxhParams {
    const float2* in;
    const unsigned* in_u8;  // U8: interleaved u8 I/Q, one dword = two samples
    long ld_in, n_in;
    const float2* hist;
    float2* hist_next;
    const float2* dummy;  // >= 1024 readable samples: target of clamped prefetches
    long n_out;
    int K;
    int delta;  // 3 - i0
    int sh;     // tap scale exponent
    const float* taps;
    float2* out;
    long ld_out;
    long tpc, spc, seg_tiles, units;  // host-checked < 2^31 (tile cursors are 32-bit)
    int ftiles;  // tiles wholly inside the input: tile t is fast iff t < ftiles (min(n_in / TI, 2^31 - 1))
    int oblk;    // 256-output blocks wholly inside the output (min(n_out / 256, 2^31 - 1))
    int vec_out;
    int blocked;  // units in per-workgroup contiguous ranges, wave w takes units w, w+8, ...
};

__device__ __forceinline__ f32x4 mfma(const u32x4& a, const u32x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ unsigned pk_rtz(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(a, b));
}

__device__ __forceinline__ float lo_f(unsigned u) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(u & 0xffffu));
}
__device__ __forceinline__ float hi_f(unsigned u) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(u >> 16));
}

// (a, b) already scaled: packed fp16 hi = rtz(x), lo = rtz(x - hi).  (Four
// v_fma_mix{lo,hi}_f16 under a round-toward-zero f16 mode give the same bytes from 4 VALU
// instead of 6 and run faster at steady state, but slower in the driver's window:
// profiles/r05_fir_ring_ab.txt F.)
__device__ __forceinline__ void split2(float a, float b, unsigned& hi, unsigned& lo) {
    hi = pk_rtz(a, b);
    lo = pk_rtz(a - lo_f(hi), b - hi_f(hi));
}

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

__device__ __forceinline__ float4 fetch_pair(const float2* in, const float2* hist, long j,
                                             long n_in, int K) {
    const float2 a = fetch1(in, hist, j, n_in, K), b = fetch1(in, hist, j + 1, n_in, K);
    return make_float4(a.x, a.y, b.x, b.y);
}

// RtlTcpSignal::next (reference src/rtltcp.rs:156-164): (v - 128) / 128, exact in f32
__device__ __forceinline__ float2 u8_iq(unsigned short w) {
    return make_float2(((float)(w & 0xffu) - 128.0f) / 128.0f, ((float)(w >> 8) - 128.0f) / 128.0f);
}
// back to the u8 code of an exactly-converted sample (history written by this handle)
__device__ __forceinline__ unsigned iq_u8(float2 v) {
    return (unsigned)(v.x * 128.0f + 128.0f) | ((unsigned)(v.y * 128.0f + 128.0f) << 8);
}
// samples (j, j+1) as one dword of u8 codes, with history / zero (code 128) fill
__device__ __forceinline__ unsigned fetch_pair_u8(const unsigned short* in, const float2* hist,
                                                  long j, long n_in, int K) {
    unsigned w = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const long q = j + e;
        const bool inb = (q >= 0) & (q < n_in);
        const bool inh = (q < 0) & (q >= -(long)(K - 1));
        const unsigned a = in[inb ? q : 0];
        const unsigned b = iq_u8(hist[inh ? q + (K - 1) : 0]);
        w |= (inb ? a : (inh ? b : 0x8080u)) << (16 * e);
    }
    return w;
}
// u8 samples are integers after the x128 scale: exact in fp16, no lo planes
template <int PLB>
__device__ __forceinline__ void put_pair_u8(char* lds, int a, unsigned w) {
    const float r0 = (float)(w & 0xffu) - 128.f, i0 = (float)((w >> 8) & 0xffu) - 128.f;
    const float r1 = (float)((w >> 16) & 0xffu) - 128.f, i1 = (float)(w >> 24) - 128.f;
    *reinterpret_cast<unsigned*>(lds + a) = pk_rtz(r0, r1);
    *reinterpret_cast<unsigned*>(lds + a + 2 * PLB) = pk_rtz(i0, i1);
}

__device__ __forceinline__ void st32(char* lds, int a, unsigned v) {
    *reinterpret_cast<unsigned*>(lds + a) = v;
}

// scale + split one sample pair into the 4 planes (re hi, re lo, im hi, im lo) at byte a
template <int PLB>
__device__ __forceinline__ void put_pair(char* lds, int a, const float4& f, float sc) {
    unsigned h, l;
    split2(f.x * sc, f.z * sc, h, l);
    st32(lds, a, h);
    st32(lds, a + PLB, l);
    split2(f.y * sc, f.w * sc, h, l);
    st32(lds, a + 2 * PLB, h);
    st32(lds, a + 3 * PLB, l);
}

// a left-leaning chain folds into two v_maximum3_f32 with |.| source modifiers: IEEE maximum,
// so a NaN sample makes the max NaN (fmaxf / v_max3_f32 would skip it; same instruction count)
__device__ __forceinline__ float absmax4(float m, const float4& f) {
    auto mx = [](float a, float b) { return __builtin_elementwise_maximum(a, b); };
    return mx(mx(mx(mx(m, fabsf(f.x)), fabsf(f.y)), fabsf(f.z)), fabsf(f.w));
}

// window scale exponent: 15 - exponent(wave max), clamped so 2^s is a normal float.  The
// wave max uses DPP row reductions (each one v_max_u32 with a DPP source) + 4 readlanes
// (non-negative floats order like their bits), and the exponent comes from the max's bits in
// scalar ops: no LDS round trips and few vector instructions on the per-tile critical path.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_umax(unsigned x) {
    const unsigned y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, true);
    return x > y ? x : y;
}
__device__ __forceinline__ int wave_scale(float m) {
    unsigned x = __float_as_uint(m);
    x = dpp_umax<0xB1>(x);   // quad_perm [1,0,3,2]
    x = dpp_umax<0x4E>(x);   // quad_perm [2,3,0,1]
    x = dpp_umax<0x141>(x);  // row_half_mirror
    x = dpp_umax<0x140>(x);  // row_mirror: every lane holds its row's max
    const unsigned a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 16);
    const unsigned c = __builtin_amdgcn_readlane(x, 32), d = __builtin_amdgcn_readlane(x, 48);
    const unsigned ab = a > b ? a : b, cd = c > d ? c : d;
    // 15 - frexp exponent = 141 - biased exponent for a normal max; a zero or subnormal max
    // (biased 0) gives 141, clamped to 126 (round 4's v_frexp_exp form gave 15 for an exact zero:
    // an all-zero window's outputs are zero either way, but the sticky-scale keep / restage
    // choice of the odd tile after it can differ, so its low bits are not round 4's); inf / NaN
    // (biased 255; absmax4 propagates NaN) -> kNonFinite: exact_tile computes that tile
    const int e = (int)((ab > cd ? ab : cd) >> 23);
    const int s = 141 - e;
    return e == 255 ? kNonFinite : (s < -126 ? -126 : (s > 126 ? 126 : s));
}

// A window holding inf or NaN (wave_scale returns kNonFinite) has no power-of-two scale, and the
// banded Toeplitz's zero taps would carry 0 x NaN = NaN into outputs whose 255-sample window does
// not hold the sample.  Such a tile's outputs come from the reference's own sum instead
// (fir.rs:28-30: acc = 0; acc += x[g - k] * h[k] for k = 0 .. K-1, no FMA; convolve.rs:13-15),
// one output per lane at a time from global memory (the tile is L2-resident), with the lanes'
// MFMA output mapping: non-finite samples reach exactly the outputs they reach in the reference,
// and the tile's finite outputs are bit-identical to it.  Only tiles that hold such a sample
// take this path.
// One f32 multiply-then-add per call, as the VOP2 instructions: the compiler would otherwise pair
// the re and im chains into v_pk_mul_f32 / v_pk_add_f32, and packed-f32 results read by the next
// packed op came out wrong (the low half, in 16-lane groups, run to run) in this wave while its
// SIMD partner ran MFMAs -- the fault of DESIGN.md 3.6, reproduced inside this kernel
// (profiles/r06_nonfinite.txt).  IEEE-exact, no contraction: the reference's `acc += x * h`.
__device__ __forceinline__ float mul_add_vop2(float acc, float x, float h) {
    float p, r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(p) : "v"(x), "v"(h));
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(acc), "v"(p));
    return r;
}

template <int D, int CS>
__device__ __forceinline__ void exact_tile(const MxhParams& p, long ch, int tile, int sv, int g) {
#pragma clang fp contract(off)
    const int K = p.K;
    const float2* __restrict__ in = p.in + ch * p.ld_in;
    const float2* __restrict__ hist = p.hist + ch * (long)(K - 1);
    float2* __restrict__ out = p.out + ch * p.ld_out;
    const long i0 = D - 1 - p.delta;
#pragma unroll 1
    for (int o = 0; o < 4 * CS; ++o) {  // column set o / 4, output o % 4 of the lane's four
        {
            const long m = (long)tile * (256 * CS) + 256 * (o >> 2) + 16 * sv + 4 * g + (o & 3);
            if (m >= p.n_out) continue;
            const long gi = i0 + (long)D * m;
            float ar = 0.f, ai = 0.f;
            if (gi - (K - 1) >= 0 && gi < p.n_in) {
                // window inside this block: 16 loads in flight per step, the sum still in k order
                // (an all-NaN stream takes this path in every tile)
                const float2* __restrict__ xp = in + gi;
                const int kb = K & ~15;
#pragma unroll 1
                for (int k = 0; k < kb; k += 16) {
                    float2 xv[16];
                    float hk[16];
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        xv[u] = xp[-(k + u)];
                        hk[u] = p.taps[k + u];
                    }
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        ar = mul_add_vop2(ar, xv[u].x, hk[u]);
                        ai = mul_add_vop2(ai, xv[u].y, hk[u]);
                    }
                }
#pragma unroll 1
                for (int k = kb; k < K; ++k) {
                    const float2 xv = xp[-k];
                    const float hk = p.taps[k];
                    ar = mul_add_vop2(ar, xv.x, hk);
                    ai = mul_add_vop2(ai, xv.y, hk);
                }
            } else {
#pragma unroll 1
                for (int k = 0; k < K; ++k) {
                    const float2 xv = fetch1(in, hist, gi - k, p.n_in, K);
                    const float hk = p.taps[k];
                    ar = mul_add_vop2(ar, xv.x, hk);
                    ai = mul_add_vop2(ai, xv.y, hk);
                }
            }
            out[m] = make_float2(ar, ai);
        }
    }
}

__device__ __forceinline__ float exp2i(int s) { return __builtin_amdgcn_ldexpf(1.0f, s); }

// Samples are streamed once: non-temporal loads and output stores.
// U8: interleaved u8 I/Q input (rtl_tcp ingest fused into the load, 2 B per sample); the
// samples are exact integers after a fixed x128 scale, so no per-tile scale, no lo planes,
// 2 MFMAs per component per chunk.
// D: decimation 4 (XOR-swizzled LDS rows, block map sigma) or 1 (linear LDS: blocks 16
// samples apart already hit distinct banks; identity block map).
template <int NCH, bool U8 = false, int D = 4, int CS = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2, 2)))
void fir_mxh_kernel(MxhParams p) {
    using Raw = std::conditional_t<U8, unsigned, float4>;
    using G = GeoH<NCH, D, CS>;
    constexpr int H = G::H, HR = G::HR, PLB = G::PLB, NH = G::NH, NG = G::NG;
    constexpr int TI = G::TI;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    claim_simd_half();  // two waves fill the SIMD: nothing else shares it (common.hpp)
    const int lane = threadIdx.x & 63;
    // wave-uniform (readfirstlane), so the tile cursors and channel addressing stay scalar
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the younger half of the workgroup (waves 4-7) loses VALU arbitration to its SIMD partner
    // on every segment (priority, then age): one static s_setprio 1 for it, no per-segment
    // flips (configs[1]: 0.5229 -> 0.5189 ms over 3 A/B reps, profiles/r02_fir_prio_ab.txt)
    if (wv >= kWaves / 2) __builtin_amdgcn_s_setprio(1);
    const long wave = (long)blockIdx.x * kWaves + wv;
    const long nwaves = (long)gridDim.x * kWaves;
    const int g = lane >> 4, v = lane & 15;
    const int K = p.K;
    const int base = wv * G::WAVE;

    // ---- A: scaled tap Toeplitz fragments (fp16 hi / lo) ----
    u32x4 ah[NCH], al[NCH];
    {
        const float tsc = exp2i(p.sh);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                unsigned hw = 0, lw = 0;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int pidx = 32 * c + 8 * g + 2 * jj + e;
                    const int k = D * v + D - 1 - p.delta + HR - pidx;
                    const bool ok = (k >= 0) & (k < K);
                    const float hk = p.taps[ok ? k : 0];
                    const float hs = ok ? hk * tsc : 0.f;
                    const _Float16 h16 = (_Float16)hs;
                    const _Float16 l16 = (_Float16)(hs - (float)h16);
                    hw |= (unsigned)__builtin_bit_cast(unsigned short, h16) << (16 * e);
                    lw |= (unsigned)__builtin_bit_cast(unsigned short, l16) << (16 * e);
                }
                ah[c][jj] = hw;
                al[c][jj] = lw;
            }
        }
    }

    const int sv = D == 4 ? sigma(v) : v;
    int rb[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if constexpr (D == 4) {
            const int r = sv + (c >> 1);
            rb[c] = base + 128 * r + 16 * ((4 * (c & 1) + g) ^ ((r >> 1) & 7));
        } else if constexpr (D == 2) {
            // 64-byte rows (32 samples), row r = v + c, 16-byte unit g ^ ((r >> 1) & 3): every
            // 16-lane group of a fragment read hits distinct banks (fir_mxi.hip's D = 4 layout)
            const int r = v + c;
            rb[c] = base + 64 * r + 16 * (g ^ ((r >> 1) & 3));
        } else {
            rb[c] = base + 2 * (G::OFF + 16 * sv + 32 * c + 8 * g);
        }
    }
    // D = 2: sample s of a 128-sample group at 64 (s >> 5) + 16 (((s >> 3) & 3) ^ ((s >> 6) & 3))
    // + 2 (s & 7); group k adds 256 k and flips unit bit 1 when k is odd
    const int wb0 = D == 4   ? base + 128 * (lane >> 5) + 4 * (lane & 3) + 16 * ((lane >> 2) & 7)
                    : D == 2 ? base + 64 * (lane >> 4) + 4 * (lane & 3) + 16 * (((lane >> 2) & 3) ^ (lane >> 5))
                             : base + 4 * lane;

    // ---- the wave's tile stream ----
    // Units (runs of seg_tiles tiles of one channel) are dealt to waves either in per-
    // workgroup contiguous ranges (p.blocked: wave w of the workgroup takes units w, w+8, ...,
    // so a CU's eight waves stream eight ADJACENT runs -- one HBM locality window per CU) or
    // grid-strided (wave b * 8 + w takes units b * 8 + w + k * 8 * grid: one chip-wide window at
    // a time).  The wave walks its units as ONE stream of tiles: three cursors (tile k
    // computed and stored, k+1 staged, k+2 loading) advance together, so the raw-tile
    // prefetch crosses run boundaries; a run's first window re-reads the H samples before it
    // (issued one tile ahead, into the history registers).
    // Cursor fields and every per-tile test are 32-bit (scalar compares; 64-bit ones are
    // vector instructions on gfx950): tile t of a channel is "fast" (its window wholly inside
    // the input) iff t < ftiles, and its outputs are whole 256-blocks iff t CS + j < oblk.
    struct Cur {
        int u, t, ch, tu, nt;
        bool ok;
    };
    const int units = (int)p.units, spc = (int)p.spc, segt = (int)p.seg_tiles, tpc = (int)p.tpc;
    const int ust = p.blocked ? kWaves : (int)nwaves;
    const int ub1 = p.blocked ? (int)(((long)blockIdx.x + 1) * p.units / gridDim.x) : units;
    auto seek = [&](Cur& c, int u) {
        c.u = u;
        c.t = 0;
        c.ok = u < ub1;
        if constexpr (D == 4 && !U8) {  // one stream (the headline): no division per unit
            c.ch = c.ok && spc < units ? u / spc : 0;
        } else {
            c.ch = c.ok ? u / spc : 0;
        }
        c.tu = (u - c.ch * spc) * segt;
        c.nt = c.ok ? std::min(segt, tpc - c.tu) : 0;
        if (c.ok && c.nt <= 0) c.ok = false;  // (units past a channel's last tile: none by construction)
    };
    auto adv = [&](Cur& c) {
        if (!c.ok) return;
        if (++c.t >= c.nt) seek(c, c.u + ust);
    };
    const long n_in = p.n_in;
    auto tile_j0 = [&](const Cur& c) { return (long)TI * (c.tu + c.t); };
    auto tile_fast = [&](const Cur& c) { return c.tu + c.t < p.ftiles; };
    auto fetch = [&](const Cur& c, long j) -> Raw {
        const float2* hist = p.hist + c.ch * (long)(K - 1);
        if constexpr (U8)
            return fetch_pair_u8(reinterpret_cast<const unsigned short*>(p.in_u8) + c.ch * p.ld_in, hist, j,
                                 n_in, K);
        else
            return fetch_pair(p.in + c.ch * p.ld_in, hist, j, n_in, K);
    };
    auto put = [&](int a, const Raw& w, float sc) {
        if constexpr (U8) put_pair_u8<PLB>(smem, a, w);
        else put_pair<PLB>(smem, a, w, sc);
    };
    // 16 B (c64 pair) or 4 B (u8 pair) per lane; j = first sample of the pair
    auto ldx = [&](const Cur& c, long j, auto nt_c) -> Raw {
        constexpr bool NT = decltype(nt_c)::value;
        if constexpr (U8) {
            const unsigned* q = p.in_u8 + c.ch * (p.ld_in / 2) + (j >> 1);
            return NT ? __builtin_nontemporal_load(q) : *q;
        } else {
            const f32x4* q = reinterpret_cast<const f32x4*>(p.in + c.ch * p.ld_in + j);
            const f32x4 r = NT ? __builtin_nontemporal_load(q) : *q;
            return make_float4(r[0], r[1], r[2], r[3]);
        }
    };
    auto load_tile = [&](Raw (&dst)[NG], const Cur& c) {
        const long j0 = tile_j0(c);
        if (tile_fast(c)) {
#pragma unroll
            for (int k = 0; k < NG; ++k) dst[k] = ldx(c, j0 + 128 * k + 2 * lane, std::true_type());
        } else {
            // stream start / end only: keep this path out of the hot loop (the clamped,
            // always-dereferenceable loads would otherwise be speculated into every tile)
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < NG; ++k) dst[k] = fetch(c, j0 + 128 * k + 2 * lane);
        }
    };
    // the H samples before tile c (plain loads: the neighbouring wave streams them too)
    auto load_hist = [&](Raw (&dst)[NH], const Cur& c) {
        const long j = tile_j0(c) - H;
        const int tile = c.tu + c.t;  // j >= 0 and j + H <= n_in (H <= TI)
        if (tile >= 1 && tile <= p.ftiles) {
#pragma unroll
            for (int k = 0; k < NH; ++k) dst[k] = ldx(c, j + 128 * k + 2 * lane, std::false_type());
        } else {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < NH; ++k) dst[k] = fetch(c, j + 128 * k + 2 * lane);
        }
    };
    auto window_scale = [&](const Raw (&nx)[NG], const Raw (&hr)[NH]) -> int {
        if constexpr (U8) {
            return 7;  // x128: the u8 codes minus 128, exact
        } else {
            float m = 0.f;
#pragma unroll
            for (int k = 0; k < NG; ++k) m = absmax4(m, nx[k]);
#pragma unroll
            for (int k = 0; k < NH; ++k) m = absmax4(m, hr[k]);
            return wave_scale(m);
        }
    };
    // byte offset of the sample pair (2 lane, 2 lane + 1) of history group k / new group k
    auto hist_addr = [&](int k) {
        if constexpr (D == 4) return (wb0 ^ (16 * (k & 7))) + 256 * k;
        else if constexpr (D == 2) return (wb0 ^ (32 * (k & 1))) + 256 * k;
        else return wb0 + 256 * k;
    };
    auto new_addr = [&](int k) {
        if constexpr (D == 4) return (wb0 ^ (16 * ((H / 128 + k) & 7))) + 128 * (H / 64 + 2 * k);
        else if constexpr (D == 2) return (wb0 ^ (32 * ((H / 128 + k) & 1))) + 2 * H + 256 * k;
        else return wb0 + 2 * H + 256 * k;
    };
    // next history = the last NH groups of (history ++ this tile's groups)
    auto roll_hist = [&](Raw (&hr)[NH], const Raw (&tile)[NG]) {
        Raw nh[NH];
#pragma unroll
        for (int i = 0; i < NH; ++i) nh[i] = NG + i < NH ? hr[(NG + i) % NH] : tile[(NG + i - NH) % NG];
#pragma unroll
        for (int i = 0; i < NH; ++i) hr[i] = nh[i];
    };

    // byte offsets of the two line-complete output stores inside a tile's first 256-block
    // (column set j adds 2048 j): the even lane of a pair writes its own 2 outputs and then
    // the odd partner's first 2, the odd lane the even partner's last 2 and then its own
    const bool ev = (v & 1) == 0;
    const unsigned om = 8u * (16 * sv + 4 * g), omp = 8u * (16 * (D == 4 ? sigma(v ^ 1) : (v ^ 1)) + 4 * g);
    const unsigned ob1 = ev ? om : omp + 16, ob2 = ev ? omp : om + 16;

    // one raw tile in flight per wave (NG <= 8 groups of registers)
    static_assert(NG <= 8 && 2 * NG > 8, "one raw tile in flight");
    static_assert(NG > NH, "an even window's last NH groups come from keep[]");
    Cur cm, st, ld;
    const int first_unit = p.blocked ? (int)((long)blockIdx.x * p.units / gridDim.x) + wv : (int)wave;
    int nf_tiles = 0;  // tiles whose window held inf / NaN (wave-uniform)
    seek(cm, first_unit);
    if (cm.ok) {
        Raw nx[NG], hr[NH];
        load_hist(hr, cm);
        load_tile(nx, cm);
        int s_cur = window_scale(nx, hr);
        {
            const float sc = exp2i(s_cur);
#pragma unroll
            for (int k = 0; k < NH; ++k) put(hist_addr(k), hr[k], sc);
#pragma unroll
            for (int k = 0; k < NG; ++k) put(new_addr(k), nx[k], sc);
        }
        st = cm;
        adv(st);
        if (st.ok && st.t == 0) load_hist(hr, st);
        else roll_hist(hr, nx);
        if (st.ok) load_tile(nx, st);
        ld = st;
        adv(ld);

        auto body = [&](auto tau_c) {
            constexpr int TAU = decltype(tau_c)::value;  // parity of tile k (computed)
            constexpr int P = 1 - TAU;                   // parity of tile k+1 (staged)
            constexpr int WN = P * G::WODD;              // staging window offset
            const bool fast2 = ld.ok && tile_fast(ld);
            const bool ld_run = ld.ok && ld.t == 0;  // tile k+2 opens a run: reload history
            // prefetch source: tile k+2, or the zeroed dummy buffer (scalar select)
            const long j2 = tile_j0(ld);
            const float2* src2 = fast2 ? p.in + ld.ch * p.ld_in + j2 : p.dummy;
            const unsigned* src2u = fast2 ? p.in_u8 + ld.ch * (p.ld_in / 2) + (j2 >> 1)
                                          : reinterpret_cast<const unsigned*>(p.dummy);
            // Sticky scale: an odd tile that continues the run of the even tile before it finds
            // its history already staged (the even window's tail) and keeps that tile's scale
            // while its window max stays within [2^7, 2^16) at it (s_fresh - s_cur in [-1, 7]:
            // no fp16 overflow; the lo parts' 2^-24 quantum stays below 2^-31 of the max).
            // Otherwise (even tiles, run starts, scale changes) the window gets its own scale
            // 2^s, s = 15 - exponent(max), and its history is staged.
            const int s_fresh = window_scale(nx, hr);
            const int dsc = s_fresh - s_cur;
            const bool keep_scale = P == 1 && st.t > 0 && dsc >= -1 && dsc <= 7;
            const int s_next = keep_scale ? s_cur : s_fresh;
            const bool hist_late = P == 1 && !keep_scale;  // odd window: history after the loop
            const float scn = exp2i(s_next);
            constexpr int NK = NG < NH ? NG : NH;  // staged groups that become history
            Raw keep[NK];
            f32x4 cr[CS], ci[CS];
#pragma unroll
            for (int j = 0; j < CS; ++j) {
                cr[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                ci[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            u32x4 fb[2][4];
            // column set j of the tile reads 256 samples (D = 1) further into the window
            auto read_frags = [&](u32x4 (&f)[4], int c, int j) {
                const int a = rb[c] + TAU * G::WODD + j * 2 * 256 * D;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (!U8 || (q & 1) == 0)
                        f[q] = *reinterpret_cast<const u32x4*>(smem + a + q * PLB);
            };
            read_frags(fb[0], 0, 0);
            // D = 1: column set j + 1's chunk 0 reads the window span of set j's last chunk
            // (256 samples = NCH - 1 chunks of 32 further), so that fragment is not re-read:
            // the slot of chunk i is (i - j) & 1
            constexpr bool kShare = D == 1 && 32 * (NCH - 1) == 256;
#pragma unroll
            for (int i = 0; i < CS * NCH; ++i) {
                const int j = i / NCH, c = i % NCH;
                {
                    const int ni = i + 1;
                    const bool reuse = kShare && ni % NCH == 0;
                    if (ni < CS * NCH && !reuse)
                        read_frags(fb[(kShare ? ni - ni / NCH : ni) & 1], ni % NCH, ni / NCH);
                    __builtin_amdgcn_sched_barrier(0);
                    const u32x4(&f)[4] = fb[(kShare ? i - j : i) & 1];
                    cr[j] = mfma(al[c], f[0], cr[j]);
                    ci[j] = mfma(al[c], f[2], ci[j]);
                    if (!U8) {
                        cr[j] = mfma(ah[c], f[1], cr[j]);
                        ci[j] = mfma(ah[c], f[3], ci[j]);
                    }
                    cr[j] = mfma(ah[c], f[0], cr[j]);
                    ci[j] = mfma(ah[c], f[2], ci[j]);
                }
                if (i == 0) {  // even window k+1's history (old hr); then tile k+2's, if it opens a run
                    if (P == 0) {
#pragma unroll
                        for (int k = 0; k < NH; ++k) put(WN + hist_addr(k), hr[k], scn);
                    }
                    if (ld_run && !hist_late) load_hist(hr, ld);
                }
#pragma unroll
                for (int k = 0; k < NG; ++k) {
                    if ((k / kStagePerChunk < CS * NCH - 1 ? k / kStagePerChunk : CS * NCH - 1) != i) continue;
                    // an even window's last NH groups overlap the odd window being read: later
                    if (P == 1 || k < NG - NH) put(WN + new_addr(k), nx[k], scn);
                    if (k >= NG - NH) keep[k - (NG > NH ? NG - NH : 0)] = nx[k];
                    if constexpr (U8) {
                        nx[k] = __builtin_nontemporal_load(src2u + 64 * k + lane);
                    } else {
                        const f32x4 r = __builtin_nontemporal_load(
                            reinterpret_cast<const f32x4*>(src2 + 128 * k + 2 * lane));
                        nx[k] = make_float4(r[0], r[1], r[2], r[3]);
                    }
                }
            }
            // after tile k's last fragment reads (same wave, LDS in order): the writes that land
            // in tile k's window
            if constexpr (P == 0) {
#pragma unroll
                for (int k = NG - NH; k < NG; ++k) put(WN + new_addr(k), keep[k - (NG - NH)], scn);
            } else {
                if (hist_late) {
#pragma unroll
                    for (int k = 0; k < NH; ++k) put(WN + hist_addr(k), hr[k], scn);
                    if (ld_run) load_hist(hr, ld);
                }
            }
            if (!ld_run) {  // history of tile k+2's window: roll in the staged tile's tail
                Raw tile[NG];
#pragma unroll
                for (int k = 0; k < NG; ++k) tile[k] = keep[k < (NG > NH ? NG - NH : 0) ? 0 : k - (NG > NH ? NG - NH : 0)];
                roll_hist(hr, tile);
            }
            if (!fast2 && ld.ok) load_tile(nx, ld);
            const int so = -(s_cur + p.sh);
            const int tile = cm.tu + cm.t;
            if (!U8 && s_cur == kNonFinite) {
                ++nf_tiles;  // its outputs come from exact_tile after the main loop
            } else {
                float2* __restrict__ out = p.out + cm.ch * p.ld_out;
                // the tile's output base is scalar; the lanes' byte offsets inside it are fixed
                char* __restrict__ outt = reinterpret_cast<char*>(out + (long)tile * G::TO);
#pragma unroll
                for (int j = 0; j < CS; ++j) {
                    float yr[4], yi[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        yr[i] = __builtin_amdgcn_ldexpf(cr[j][i], so);
                        yi[i] = __builtin_amdgcn_ldexpf(ci[j][i], so);
                    }
                    if (p.vec_out && tile * CS + j < p.oblk) {
                        // line-complete stores: lanes v and v^1 (same g) swap one 16-B half, so the
                        // first store writes the 128-B lines of the even-v blocks whole (8 lanes per
                        // line) and the second those of the odd-v blocks (steady-state probe: 0.472
                        // vs 0.487 ms for half-line pairs, profiles/r03s3_stream_probe3.txt)
                        const f32x4 y0 = {yr[0], yi[0], yr[1], yi[1]};
                        const f32x4 y1 = {yr[2], yi[2], yr[3], yi[3]};
                        f32x4 rx;
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            rx[q] = __int_as_float(__builtin_amdgcn_mov_dpp(
                                __float_as_int(ev ? y1[q] : y0[q]), 0xB1, 0xf, 0xf, false));
                        __builtin_nontemporal_store(ev ? y0 : rx, reinterpret_cast<f32x4*>(outt + (ob1 + 2048u * j)));
                        __builtin_nontemporal_store(ev ? rx : y1, reinterpret_cast<f32x4*>(outt + (ob2 + 2048u * j)));
                    } else {
                        const long m = (long)tile * G::TO + 256 * j + 16 * sv + 4 * g;  // sv = block of column v
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (m + i < p.n_out) out[m + i] = make_float2(yr[i], yi[i]);
                    }
                }
            }
            s_cur = s_next;
            cm = st;
            st = ld;
            adv(ld);
        };
        // two tiles per iteration: the window ring half is compile-time in every body
        while (cm.ok) {
            body(std::integral_constant<int, 0>());
            if (!cm.ok) break;
            body(std::integral_constant<int, 1>());
        }
    }
    if constexpr (!U8) {
        // the tiles the loop skipped: walk the wave's tiles again and give every one whose
        // window [j0 - H, j0 + TI) holds inf / NaN (exactly those whose scale was kNonFinite)
        // the reference's sums -- out of the main loop, so its code leaves the loop's
        // registers and schedule alone
        if (nf_tiles > 0) {
            Cur c;
            seek(c, first_unit);
            while (c.ok) {
                const long j0 = tile_j0(c) - H;
                bool bad = false;
                for (int q = lane; q < H + TI; q += 64) {
                    const float2 xv = fetch1(p.in + c.ch * p.ld_in, p.hist + c.ch * (long)(K - 1),
                                             j0 + q, n_in, K);
                    bad |= !(__builtin_isfinite(xv.x) && __builtin_isfinite(xv.y));
                }
                if (__builtin_amdgcn_ballot_w64(bad) != 0) exact_tile<D, CS>(p, c.ch, c.tu + c.t, sv, g);
                adv(c);
            }
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
            if constexpr (U8) {
                const unsigned short* inb = reinterpret_cast<const unsigned short*>(p.in_u8) + ch * p.ld_in;
                p.hist_next[j] = gidx >= 0 ? u8_iq(inb[gidx]) : hic[gidx + (K - 1)];
            } else {
                p.hist_next[j] = gidx >= 0 ? inc[gidx] : hic[gidx + (K - 1)];
            }
        }
    }
}

int mxh_nch(int K, int D) {
    if (D == 4) {
        const int need = (K + 63 + 31) / 32;  // 32 NCH >= K + 15*4 + 3
        return need <= 6 ? 6 : (need <= 10 ? 10 : 0);
    }
    if (D == 1) {
        const int need = (K + 15 + 31) / 32;  // 32 NCH >= K + 15
        return need <= 5 ? 5 : (need <= 9 ? 9 : 0);
    }
    if (D == 2) {
        const int need = (K + 31 + 31) / 32;  // 32 NCH >= K + 15*2 + 1
        return need <= 5 ? 5 : (need <= 9 ? 9 : 0);
    }
    return 0;
}

}  // namespace

size_t fir_mxh_dummy_bytes() { return 1024 * sizeof(float2); }  // one D = 4 tile of samples

int fir_mxh_shape_ok(int sample_kind, int tap_kind, int K, int D) {
    if (tap_kind != SDRGPU_F32 || K < 1) return 0;
    if (sample_kind == SDRGPU_CU8) return D == 4 && mxh_nch(K, 4) > 0;
    return sample_kind == SDRGPU_C64 && mxh_nch(K, D) > 0;
}

int fir_mxh_supported(const FirParams& fp) {
    const bool u8 = fp.sample_kind == SDRGPU_CU8;
    if ((!u8 && fp.sample_kind != SDRGPU_C64) || fp.tap_kind != SDRGPU_F32) return 0;
    if (!(fp.D == 4 || ((fp.D == 1 || fp.D == 2) && !u8))) return 0;
    if (fp.K < 1 || mxh_nch(fp.K, fp.D) == 0) return 0;
    if (fp.i0 < 0 || fp.i0 >= fp.D) return 0;
    // 16-byte (c64) / 4-byte (u8) loads of sample pairs: channel bases stay aligned
    const uintptr_t align = u8 ? 3 : 15;
    if ((reinterpret_cast<uintptr_t>(fp.in) & align) != 0 || (fp.nch > 1 && (fp.ld_in & 1)))
        return 0;
    return 1;
}

int fir_mxh_launch(const FirParams& fp, const float* d_taps, int tap_scale_exp,
                   const void* d_dummy, int cus, hipStream_t s) {
    if (!fir_mxh_supported(fp) || !d_dummy) return SDRGPU_ERR_UNSUPPORTED;
    const int D = fp.D;
    const int NCH = mxh_nch(fp.K, D);
    MxhParams p;
    const bool u8 = fp.sample_kind == SDRGPU_CU8;
    p.in = static_cast<const float2*>(fp.in);
    p.in_u8 = static_cast<const unsigned*>(fp.in);
    p.ld_in = fp.ld_in;
    p.n_in = fp.n_in;
    p.hist = static_cast<const float2*>(fp.hist);
    p.hist_next = fp.K > 1 ? static_cast<float2*>(fp.hist_next) : nullptr;
    p.dummy = static_cast<const float2*>(d_dummy);
    p.n_out = fp.n_out;
    p.K = fp.K;
    p.delta = (int)(D - 1 - fp.i0);
    p.sh = tap_scale_exp;
    p.taps = d_taps;
    p.out = static_cast<float2*>(fp.out);
    p.ld_out = fp.ld_out;
    p.vec_out = ((reinterpret_cast<uintptr_t>(fp.out) & 15) == 0 &&
                 (fp.nch == 1 || !(fp.ld_out & 1)))
                    ? 1
                    : 0;
    const long nch = fp.nch;
    const int cs = D == 1 ? kCs1 : (D == 2 ? kCs2 : 1);
    p.tpc = ceil_div(std::max(0L, fp.n_out), 256L * cs);
    const long W = (long)kWaves * cus;
    // D = 4: runs of kRunTiles tiles (c64: grid-strided; u8: per-CU blocks, round 2: 0.516-0.525
    // vs 0.556-0.559 ms with one long range per wave, profiles/r02_fir_runs.txt).  D = 1 banks
    // keep whole-channel units grid-strided (runs measured no faster there).
    const int run = D == 4 ? (u8 ? kRunTilesU8 : kRunTiles) : (D == 2 ? kRunTiles : 0);
    long spc = nch >= W ? 1 : ceil_div(W, nch);
    spc = std::max(1L, std::min(spc, p.tpc));
    p.seg_tiles = std::max(1L, ceil_div(p.tpc, spc));
    if (run > 0) p.seg_tiles = std::max(1L, std::min<long>(run, p.tpc));
    p.spc = std::max(1L, ceil_div(p.tpc, p.seg_tiles));
    p.units = nch * p.spc;
    p.blocked = run > 0 && u8;
    const long TI = 256L * cs * D;
    p.ftiles = (int)std::min<long>(fp.n_in / TI, INT_MAX);
    p.oblk = (int)std::min<long>(std::max(0L, fp.n_out) / 256, INT_MAX);
    // 32-bit tile cursors (units, tiles per channel, unit / tile indices)
    if (p.units >= INT_MAX - 8L * cus || p.tpc >= INT_MAX) return SDRGPU_ERR_UNSUPPORTED;
    const long blocks = std::max(1L, std::min((long)cus, ceil_div(p.units, kWaves)));
#define SDRGPU_MXH_GO(CC, U, DD, CS)                                                           \
    hipLaunchKernelGGL((fir_mxh_kernel<CC, U, DD, CS>), dim3(blocks), dim3(kBlock),            \
                       (size_t)kWaves * (GeoH<CC, DD, CS>::WAVE), s, p)
#define SDRGPU_MXH_CASE(CC)                                                                    \
    if (D == 4 && NCH == CC) {                                                                 \
        if (u8) SDRGPU_MXH_GO(CC, true, 4, 1);                                                 \
        else SDRGPU_MXH_GO(CC, false, 4, 1);                                                   \
        SDRGPU_LAUNCH_CHECK();                                                                 \
        return SDRGPU_OK;                                                                      \
    }
#define SDRGPU_MXH_CASE1(CC)                                                                   \
    if (D == 1 && NCH == CC) {                                                                 \
        SDRGPU_MXH_GO(CC, false, 1, kCs1);                                                     \
        SDRGPU_LAUNCH_CHECK();                                                                 \
        return SDRGPU_OK;                                                                      \
    }
#define SDRGPU_MXH_CASE2(CC)                                                                   \
    if (D == 2 && NCH == CC) {                                                                 \
        SDRGPU_MXH_GO(CC, false, 2, kCs2);                                                     \
        SDRGPU_LAUNCH_CHECK();                                                                 \
        return SDRGPU_OK;                                                                      \
    }
    SDRGPU_MXH_CASE(10)
    SDRGPU_MXH_CASE(6)
    SDRGPU_MXH_CASE1(9)
    SDRGPU_MXH_CASE1(5)
    SDRGPU_MXH_CASE2(9)
    SDRGPU_MXH_CASE2(5)
#undef SDRGPU_MXH_CASE
#undef SDRGPU_MXH_CASE1
#undef SDRGPU_MXH_CASE2
#undef SDRGPU_MXH_GO
    return SDRGPU_ERR_UNSUPPORTED;
}

}  // namespace sdrgpu
