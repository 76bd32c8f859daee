// fir_mfma.hip -- direct-form FIR / FIR-decimate on the matrix cores (gfx950 MFMA).
//
// Same semantics as fir_direct.hip / fir_os.hip: Fir::apply + Decimate (reference
// src/filter/fir.rs:23-32, src/filter/convolve.rs:13-15, src/signal/adapters/mod.rs:30-37)
// for complex samples and real taps, y[m] = sum_k h[k] x[i0 + mD - k].
//
// Why.  The direct form needs 2K FMA per kept complex output; on the f32 VALU (and the
// f32 MFMA, which runs at the same rate) that is 34 G FMA for configs[1], > 0.7 ms at the
// clock an FMA-dense kernel holds -- far above the 0.34-0.45 ms HBM time of the stream.
// bf16 MFMA runs 16x faster, and f32 accuracy survives an EXACT three-way split:
//   x = xh + xm + xl  (xh = x with the low 16 mantissa bits cleared, xm likewise of x-xh,
//                      xl = x-xh-xm; every piece is a bf16 and the sum is exact),
//   h = hh + hm + hl  (same split of the taps),
//   x*h ~= xh*hh + xh*hm + xm*hh + xh*hl + xm*hm + xl*hh        (6 bf16 MFMAs)
// the dropped terms are < 2^-23 |x h|, and bf16 keeps f32's exponent range, so the
// result is f32-accurate for every input range (measured against the oracle: tests).
//
// GEMM shape (v_mfma_f32_16x16x32_bf16, C[16x16] += A[16x32] B[32x16]):
//   rows    u = 16 independent SEGMENTS of the stream (each a long run of outputs),
//   columns v = 16 consecutive kept outputs of one step of a segment,
//   K       = 32-sample chunks of the input window of the step:
//             A[u][k] = x[window_u + k] (data, re and im as two A's), B[k][v] = h[tap(k,v)]
// B is a banded Toeplitz of the taps, identical for every segment and step, so it lives
// in registers for the whole launch (3 splits x NCH chunks x 4 VGPRs).  A step advances a
// segment by 16 outputs = 16D input samples = D/2 chunks; the window holds NCH chunks, so
// every new chunk is multiplied ONCE into the NACC = NCH/(D/2) accumulators of the steps
// that will use it (chunk positions NCH-D/2.., then D/2 lower per later step) and then
// dropped: no data re-read, no LDS at all.  Each lane loads its A fragment straight from
// HBM: the 4 lanes of a segment read 64 contiguous bytes per instruction (the chunk's k
// order is permuted to make that so; B uses the same permutation).
//
// One wave per SIMD (~400 VGPRs: taps, 5-deep register prefetch ring, accumulators);
// 16 segments per wave, one 256-lane workgroup per CU.  Algorithmic bytes per input sample
// at D=4: 8 in + 2 out = 10 B; MFMA work 6 x (K+15D rounded to 32) / (16 x 16) per output.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "fir_exact.hpp"
#include "fir_mxi.hpp"

namespace sdrgpu {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMxBlock = 256;  // 4 waves: one per SIMD

struct MxParams {
    const float2* in;
    long ld_in, n_in;
    const float2* hist;
    float2* hist_next;
    long i0, n_out;
    int K;
    const float* taps;   // device, natural order, K f32
    int delta;           // window end alignment (makes every 16-B load aligned)
    long seg_len;        // outputs per segment (multiple of 16)
    long nseg_ch;        // segments per channel
    long nseg;           // nch * nseg_ch
    float2* out;
    long ld_out;
    int n_iter;          // iterations per segment (multiple of NACC)
    int D, tpp;          // for fir_exact_output (polyphase taps_pm)
    const void* taps_pm;
};

// A non-finite MFMA output came from an inf / NaN sample in its step's window, which the zero
// taps of the Toeplitz carry to all 16 outputs of the step.  The main loop only notes that a lane
// stored one (its registers are full); afterwards the lane re-reads its own outputs (rows 4g + i,
// column v of every step: same-thread read-after-write) and replaces the non-finite ones with
// the reference's sum (fir_exact.hpp).
__device__ __forceinline__ void mx_exact_fixup(const MxParams& p, long wave, int g, int v) {
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        const long sg = wave * 16 + 4 * g + i;
        if (sg >= p.nseg) break;
        const long ch = sg / p.nseg_ch;
        const long m = (sg - ch * p.nseg_ch) * p.seg_len;
        const long rem = p.n_out - m, lim = rem < p.seg_len ? rem : p.seg_len;
        float2* __restrict__ out = p.out + ch * p.ld_out + m;
#pragma unroll 1
        for (long o = v; o < lim; o += 16)
            if (!all_finite(out[o]))
                out[o] = fir_exact_output<float2, float>(p, p.in + ch * p.ld_in,
                                                         p.hist + ch * (long)(p.K - 1), m + o);
    }
}

// Split a pair of floats into three packed bf16 pairs (a -> low half, b -> high half):
// hi = top 16 bits, mid = top 16 bits of the exact remainder, lo = the rest (exact).
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

template <int D, int NCH>
__global__ __launch_bounds__(kMxBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fir_mx_kernel(MxParams p) {
    constexpr int NC = D / 2;         // new 32-sample chunks per step
    constexpr int NACC = NCH / NC;    // steps every chunk contributes to
    constexpr int NP = 4 * NC;        // 16-byte pieces per lane per step
    static_assert(D % 2 == 0 && NCH % NC == 0, "geometry");

    claim_simd_whole();  // one wave per SIMD, alone on it (common.hpp)
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * (kMxBlock / 64) + (threadIdx.x >> 6);
    const int g = lane >> 4, v = lane & 15;
    const int K = p.K;

    // ---- B: tap Toeplitz fragments, B[k = 8g + j][v] for chunk position c ----
    // element j <-> chunk sample pi = 8(j>>1) + 2g + (j&1); output v of the step has
    // full-rate index E - 1 - (15 - v) D (E = window end), the sample E - 32(NCH-c) + pi
    u32x4 bh[NCH], bm[NCH], bl[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            float hv[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int pi = 8 * jj + 2 * g + e;
                const int k = 32 * (NCH - c) - pi - 1 - (15 - v) * D - p.delta;
                const bool ok = (k >= 0) & (k < K);
                const float hk = p.taps[ok ? k : 0];
                hv[e] = ok ? hk : 0.f;
            }
            unsigned h, m, l;
            split3(hv[0], hv[1], h, m, l);
            bh[c][jj] = h;
            bm[c][jj] = m;
            bl[c][jj] = l;
        }
    }

    // ---- the segment this lane loads for (A row u = v) ----
    long segA = wave * 16 + v;
    if (segA >= p.nseg) segA = p.nseg - 1;  // idle rows alias a real segment (no stores)
    const long chA = segA / p.nseg_ch;
    const long mA = (segA - chA * p.nseg_ch) * p.seg_len;
    const float2* __restrict__ inA = p.in + chA * p.ld_in;
    const float2* __restrict__ hiA = p.hist + chA * (long)(K - 1);
    // first sample of the lane's first piece at iteration 0 (step t = 1 - NACC):
    // window end E_t = i0 + (m + 16t + 15) D + 1 + delta, new data [E_t - 16D, E_t)
    const long s0 = p.i0 + (mA + 16L * (1 - NACC) + 15) * D + 1 + p.delta - 16L * D + 2 * g;
    const long n_in = p.n_in;

    // ---- the 4 segments this lane stores for (C rows 4g + i) ----
    float2* outp[4];
    long lim[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const long sg = wave * 16 + 4 * g + i;
        const long sgc = sg < p.nseg ? sg : p.nseg - 1;
        const long ch = sgc / p.nseg_ch;
        const long m = (sgc - ch * p.nseg_ch) * p.seg_len;
        outp[i] = p.out + ch * p.ld_out + m + v;
        const long rem = p.n_out - m;
        lim[i] = sg < p.nseg ? (rem < p.seg_len ? rem : p.seg_len) : 0;
    }

    auto load_step = [&](float4 (&dst)[NP], long s) {
        const bool ok = (s >= 0) & (s + 32 * (NC - 1) + 26 <= n_in);
        if (__all(ok)) {
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    dst[4 * c + i] = *reinterpret_cast<const float4*>(inA + s + 32 * c + 8 * i);
        } else {
            // stream start (history), end of input (zeros), idle rows: branch-free selects
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float2 x2[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const long a = s + 32 * c + 8 * i + e;
                        const bool inb = (a >= 0) & (a < n_in);
                        const bool inh = (a < 0) & (a >= -(long)(K - 1));
                        const float2 xa = inA[inb ? a : 0];
                        const float2 xb = hiA[inh ? a + (K - 1) : 0];
                        x2[e] = inb ? xa : (inh ? xb : make_float2(0.f, 0.f));
                    }
                    dst[4 * c + i] = make_float4(x2[0].x, x2[0].y, x2[1].x, x2[1].y);
                }
        }
    };

    f32x4 accr[NACC], acci[NACC];
#pragma unroll
    for (int a = 0; a < NACC; ++a) {
        accr[a] = f32x4{0.f, 0.f, 0.f, 0.f};
        acci[a] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float4 raw[NACC][NP];
    bool nonfinite = false;    // this lane stored a non-finite output (mx_exact_fixup)
    const long hop = 16L * D;  // input samples per step
#pragma unroll
    for (int r = 0; r < NACC; ++r)
        if (r < p.n_iter) load_step(raw[r], s0 + hop * r);

#pragma unroll 1
    for (int q0 = 0; q0 < p.n_iter; q0 += NACC) {
#pragma unroll
        for (int r = 0; r < NACC; ++r) {
            const int it = q0 + r;
            // ---- split the step's new samples into bf16 fragments: [chunk][re, im] ----
            u32x4 xh[NC][2], xm[NC][2], xl[NC][2];
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float4 f = raw[r][4 * c + i];
                    unsigned h, m, l;
                    split3(f.x, f.z, h, m, l);
                    xh[c][0][i] = h;
                    xm[c][0][i] = m;
                    xl[c][0][i] = l;
                    split3(f.y, f.w, h, m, l);
                    xh[c][1][i] = h;
                    xm[c][1][i] = m;
                    xl[c][1][i] = l;
                }
            // ---- prefetch the samples of iteration it + NACC into the freed buffer ----
            if (it + NACC < p.n_iter) load_step(raw[r], s0 + hop * (it + NACC));

            {
                // ---- multiply the new chunks into the NACC pending steps ----
#pragma unroll
                for (int d = 0; d < NACC; ++d) {
                    const int slot = (r + 1 + d) % NACC;
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        const int pos = NCH - NC + c - d * NC;
                        f32x4 ar = accr[slot], ai = acci[slot];
                        ar = mfma(xl[c][0], bh[pos], ar);
                        ai = mfma(xl[c][1], bh[pos], ai);
                        ar = mfma(xm[c][0], bm[pos], ar);
                        ai = mfma(xm[c][1], bm[pos], ai);
                        ar = mfma(xh[c][0], bl[pos], ar);
                        ai = mfma(xh[c][1], bl[pos], ai);
                        ar = mfma(xm[c][0], bh[pos], ar);
                        ai = mfma(xm[c][1], bh[pos], ai);
                        ar = mfma(xh[c][0], bm[pos], ar);
                        ai = mfma(xh[c][1], bm[pos], ai);
                        ar = mfma(xh[c][0], bh[pos], ar);
                        ai = mfma(xh[c][1], bh[pos], ai);
                        accr[slot] = ar;
                        acci[slot] = ai;
                    }
                }
            }
            // ---- step t = it - (NACC - 1) is complete: store, recycle its accumulators ----
            const int slot = (r + 1) % NACC;
            const long t = (long)it - (NACC - 1);
            if (t >= 0) {
                const long o = 16 * t;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    nonfinite |= !all_finite(make_float2(accr[slot][i], acci[slot][i]));
                    if (o + v < lim[i]) outp[i][o] = make_float2(accr[slot][i], acci[slot][i]);
                }
            }
            accr[slot] = f32x4{0.f, 0.f, 0.f, 0.f};
            acci[slot] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    if (nonfinite) mx_exact_fixup(p, wave, g, v);

    if (p.hist_next) {  // stream history carry, spread over the whole grid
        const long nch = (p.nseg + p.nseg_ch - 1) / p.nseg_ch;
        for (long j = (long)blockIdx.x * kMxBlock + threadIdx.x; j < nch * (K - 1);
             j += (long)gridDim.x * kMxBlock) {
            const long ch = j / (K - 1), jj = j - ch * (K - 1);
            const float2* inc = p.in + ch * p.ld_in;
            const float2* hic = p.hist + ch * (long)(K - 1);
            const long gidx = p.n_in - (long)(K - 1) + jj;
            p.hist_next[j] = gidx >= 0 ? inc[gidx] : hic[gidx + (K - 1)];
        }
    }
}

struct MxState {
    int K = 0, D = 0, NCH = 0;
    float* d_taps = nullptr;
    void* d_dummy = nullptr;  // zeroed target of fir_mxh's clamped prefetches
    int tap_scale_exp = 0;    // fir_mxh: 15 - exponent(max |h|)
    bool taps_finite = true;  // fir_mxi takes integer taps: finite ones only
    int cus = 256;
};

int mx_nch(int K, int D) {
    if (!(D == 2 || D == 4 || D == 8)) return 0;
    // smallest instantiated chunk count covering the K + 15D + 1 window
    const int need = (K + 15 * D + 1 + 31) / 32;
    static const int c2[] = {4, 9}, c4[] = {4, 10}, c8[] = {4, 12};
    const int* c = D == 2 ? c2 : D == 4 ? c4 : c8;
    const int n = 2;
    for (int i = 0; i < n; ++i)
        if (c[i] >= need) return c[i];
    return 0;
}

}  // namespace

int fir_mx_supported(int sample_kind, int tap_kind, int K, int D) {
    if (fir_mxh_shape_ok(sample_kind, tap_kind, K, D)) return 1;
    if (sample_kind != SDRGPU_C64 || tap_kind != SDRGPU_F32) return 0;
    if (!(D == 2 || D == 4 || D == 8) || K < 1) return 0;
    return mx_nch(K, D) > 0;
}

void* fir_mx_prepare(int device, const float* taps, int K, int D, int* status) {
    if (!fir_mx_supported(SDRGPU_C64, SDRGPU_F32, K, D)) {
        if (status) *status = SDRGPU_ERR_UNSUPPORTED;
        return nullptr;
    }
    auto* st = new MxState();
    st->K = K;
    st->D = D;
    st->NCH = mx_nch(K, D);
    {
        float hmax = 0.f;
        for (int k = 0; k < K; ++k) {
            hmax = std::max(hmax, std::fabs(taps[k]));
            if (!std::isfinite(taps[k])) st->taps_finite = false;
        }
        int e = 0;
        (void)std::frexp(hmax, &e);
        st->tap_scale_exp = std::min(126, std::max(-126, 15 - e));
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        st->cus = cus;
    if (hipMalloc(&st->d_taps, sizeof(float) * K) != hipSuccess ||
        hipMemcpy(st->d_taps, taps, sizeof(float) * K, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&st->d_dummy, fir_mxh_dummy_bytes()) != hipSuccess ||
        hipMemset(st->d_dummy, 0, fir_mxh_dummy_bytes()) != hipSuccess) {
        if (st->d_taps) (void)hipFree(st->d_taps);
        if (st->d_dummy) (void)hipFree(st->d_dummy);
        delete st;
        if (status) *status = SDRGPU_ERR_NOMEM;
        return nullptr;
    }
    if (status) *status = SDRGPU_OK;
    return st;
}

void fir_mx_release(void* state) {
    auto* st = static_cast<MxState*>(state);
    if (!st) return;
    if (st->d_taps) (void)hipFree(st->d_taps);
    if (st->d_dummy) (void)hipFree(st->d_dummy);
    delete st;
}

int fir_mx_launch(const FirParams& fp, void* state, hipStream_t s, int* kernel) {
    int dummy_kernel = 0;
    int& kern = kernel ? *kernel : dummy_kernel;
    auto* st = static_cast<MxState*>(state);
    if (st && fp.sample_kind == SDRGPU_CU8) {  // rtl_tcp u8 ingest fused into the FIR load
        if (fp.D != st->D || fp.K != st->K) return SDRGPU_ERR_UNSUPPORTED;
        // the int8-MFMA kernel (16-byte aligned channels), else the fp16 one (4-byte aligned)
        if (st->taps_finite && fir_mxi_supported(fp, st->tap_scale_exp)) {
            kern = SDRGPU_FIR_KERNEL_INT8;
            return fir_mxi_launch(fp, st->d_taps, st->tap_scale_exp, st->d_dummy, st->cus, s);
        }
        if (!fir_mxh_supported(fp)) return SDRGPU_ERR_UNSUPPORTED;
        kern = SDRGPU_FIR_KERNEL_FP16;
        return fir_mxh_launch(fp, st->d_taps, st->tap_scale_exp, st->d_dummy, st->cus, s);
    }
    if (!st || fp.sample_kind != SDRGPU_C64 || fp.tap_kind != SDRGPU_F32 || fp.D != st->D ||
        fp.K != st->K)
        return SDRGPU_ERR_UNSUPPORTED;
    // D = 4, 2 and 1: the LDS-staged fp16 two-way split at two waves per SIMD (fir_mxh.hip);
    // D = 8 (and D = 2 blocks the fp16 kernel does not take): the register-fed exact bf16
    // three-way split below
    if (fir_mxh_supported(fp)) {
        kern = SDRGPU_FIR_KERNEL_FP16;
        return fir_mxh_launch(fp, st->d_taps, st->tap_scale_exp, st->d_dummy, st->cus, s);
    }
    if (st->NCH == 0) return SDRGPU_ERR_UNSUPPORTED;  // shape only the fp16 kernel covers
    // 16-byte loads of sample pairs: channel bases must stay 16-byte aligned
    if ((reinterpret_cast<uintptr_t>(fp.in) & 15) != 0 || (fp.nch > 1 && (fp.ld_in & 1)))
        return SDRGPU_ERR_UNSUPPORTED;
    const int D = st->D, NCH = st->NCH, NACC = NCH / (D / 2);
    MxParams p;
    p.in = static_cast<const float2*>(fp.in);
    p.ld_in = fp.ld_in;
    p.n_in = fp.n_in;
    p.hist = static_cast<const float2*>(fp.hist);
    p.hist_next = fp.K > 1 ? static_cast<float2*>(fp.hist_next) : nullptr;
    p.i0 = fp.i0;
    p.n_out = fp.n_out;
    p.K = fp.K;
    p.taps = st->d_taps;
    // window end E = i0 + (m + 16t + 15) D + 1 has the parity of i0 + 1 (D even, m % 16 = 0)
    p.delta = (int)((fp.i0 + 1) & 1);
    p.out = static_cast<float2*>(fp.out);
    p.ld_out = fp.ld_out;
    p.D = D;
    p.tpp = fp.tpp;
    p.taps_pm = fp.taps_pm;
    // segments: one wave per SIMD chip-wide, 16 segments per wave
    const long target = 16L * 4 * st->cus;
    const long total = fp.n_out * (long)fp.nch;
    long seg = ceil_div(std::max(1L, total), target);
    seg = std::max(64L, ceil_div(seg, 16) * 16);
    p.seg_len = seg;
    p.nseg_ch = std::max(1L, ceil_div(fp.n_out, seg));
    p.nseg = p.nseg_ch * fp.nch;
    const long steps = fp.n_out > 0 ? seg / 16 : 0;
    p.n_iter = fp.n_out > 0 ? (int)(ceil_div(steps + NACC - 1, NACC) * NACC) : 0;
    const long waves = ceil_div(p.nseg, 16);
    dim3 grid((unsigned)std::max(1L, ceil_div(waves, kMxBlock / 64)));
#define SDRGPU_MX_CASE(DD, CC)                                                                   \
    if (D == DD && NCH == CC) {                                                                  \
        kern = SDRGPU_FIR_KERNEL_BF16X3;                                                         \
        hipLaunchKernelGGL((fir_mx_kernel<DD, CC>), grid, dim3(kMxBlock), 0, s, p);                \
        SDRGPU_LAUNCH_CHECK();                                                                   \
        return SDRGPU_OK;                                                                        \
    }
    SDRGPU_MX_CASE(4, 10)
    SDRGPU_MX_CASE(4, 4)
    SDRGPU_MX_CASE(2, 4)
    SDRGPU_MX_CASE(2, 9)
    SDRGPU_MX_CASE(8, 4)
    SDRGPU_MX_CASE(8, 12)
#undef SDRGPU_MX_CASE
    return SDRGPU_ERR_UNSUPPORTED;
}

}  // namespace sdrgpu
