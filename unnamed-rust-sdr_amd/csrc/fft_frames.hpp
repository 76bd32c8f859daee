// fft_frames.hpp -- frame sources and output collation shared by the FFT kernels
// (power-of-two tiles / four-step in fft.hip, mixed-radix and Bluestein in fft_gen.hip).
#pragma once

#include "common.hpp"

namespace sdrgpu {

// -------- frame sources ---------------------------------------------------------------
struct FrameSrc {
    // mode 0: contiguous frames (frame f at in + f*M)
    // mode 1: STFT frames from a stream: frame f covers stream [f0 + (f+1)hop - M, +M), stream
    //         index g < 0 -> hist[g + H] (H = history length) if g >= -H, else 0; g >= n_in -> 0
    // mode 2: contiguous REAL frames (float, imag = 0) -- rfft
    // mode 3: as mode 1 from an rtl_tcp u8 I/Q stream (RtlTcpSignal::next, src/rtltcp.rs:156-164,
    //         converted in the load: (v - 128) / 128); the history stays C64
    int mode;
    const float2* in;
    const float* in_real;
    const unsigned short* in_u8;
    long n_in;
    const float2* hist;
    long H;
    long first_end;  // stream index (exclusive end) of frame 0 of this launch
    long hop;
};

__host__ __device__ inline bool frame_src_is_stream(int mode) { return mode == 1 || mode == 3; }

__device__ __forceinline__ float2 u8_sample(unsigned short w) {
    return make_float2(((float)(w & 0xffu) - 128.0f) / 128.0f, ((float)(w >> 8) - 128.0f) / 128.0f);
}

__device__ __forceinline__ float2 frame_sample(const FrameSrc& s, long M, long f, long n) {
    if (s.mode == 0) return s.in[f * M + n];
    if (s.mode == 2) return make_float2(s.in_real[f * M + n], 0.f);
    const long g = s.first_end + f * s.hop - M + n;
    if (g >= 0) {
        if (g >= s.n_in) return make_float2(0.f, 0.f);
        return s.mode == 3 ? u8_sample(s.in_u8[g]) : s.in[g];
    }
    if (g >= -s.H) return s.hist[g + s.H];
    return make_float2(0.f, 0.f);
}

// Workgroup-uniform fast gather: when frames [f0, f0 + nf) of a workgroup lie wholly inside
// the input (no history, no zero fill), sample (f, n) of them is base[f * stride + n] with
// one load type, so a tile's loads can all be in flight at once (frame_sample's per-mode,
// per-range branches put a vmcnt wait between consecutive loads).
struct FrameFast {
    int kind;  // 0: use frame_sample; 1: c64, 2: real f32, 3: rtl_tcp u8 pairs
    const float2* c;
    const float* r;
    const unsigned short* u;
    long stride;  // samples between consecutive frames
};

__device__ __forceinline__ FrameFast frame_fast(const FrameSrc& s, long M, long f0, long nf) {
    FrameFast q{0, nullptr, nullptr, nullptr, M};
    if (nf <= 0) return q;
    if (s.mode == 0) {
        q.kind = 1;
        q.c = s.in + f0 * M;
    } else if (s.mode == 2) {
        q.kind = 2;
        q.r = s.in_real + f0 * M;
    } else {
        const long g0 = s.first_end + f0 * s.hop - M, g1 = s.first_end + (f0 + nf - 1) * s.hop;
        if (g0 >= 0 && g1 <= s.n_in) {
            q.kind = s.mode == 3 ? 3 : 1;
            q.stride = s.hop;
            if (s.mode == 3) q.u = s.in_u8 + g0;
            else q.c = s.in + g0;
        }
    }
    return q;
}

// PER samples per lane, lane-strided over the tile (p = t + BLK u, frame p / M via div):
// v[u] = sample of point p, or 0 past the tile / the last frame
template <int PER, int BLK, typename Div>
__device__ __forceinline__ void gather_tile(const FrameSrc& s, long M, long f0, int nf, int L,
                                            const Div& div, float2 (&v)[PER]) {
    const FrameFast q = frame_fast(s, M, f0, nf);
    const int t = threadIdx.x;
    if ((q.kind == 1 || q.kind == 3) && nf * M == L && (nf - 1) * q.stride + M < (1L << 28)) {
        // every frame of the tile present and inside the input: point p = f M + n sits at
        // sample p + f (stride - M) of the first frame, a 32-bit byte offset off a scalar base
        const int d = (int)(q.stride - M);
        if (q.kind == 1) {
            const char* base = reinterpret_cast<const char*>(q.c);
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int p = t + u * BLK;
                const unsigned off = (unsigned)(p + div(p) * d) * 8u;
                v[u] = p < L ? *reinterpret_cast<const float2*>(base + off) : make_float2(0.f, 0.f);
            }
        } else {
            const char* base = reinterpret_cast<const char*>(q.u);
            unsigned short w[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int p = t + u * BLK;
                const unsigned off = (unsigned)(p + div(p) * d) * 2u;
                w[u] = p < L ? *reinterpret_cast<const unsigned short*>(base + off) : (unsigned short)0x8080;
            }
#pragma unroll
            for (int u = 0; u < PER; ++u) v[u] = u8_sample(w[u]);
        }
        return;
    }
    if (q.kind == 1) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = t + u * BLK, f = div(p), n = p - f * (int)M;
            const bool ok = p < L && f < nf;
            const float2 x = q.c[ok ? f * q.stride + n : 0];
            v[u] = ok ? x : make_float2(0.f, 0.f);
        }
    } else if (q.kind == 2) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = t + u * BLK, f = div(p), n = p - f * (int)M;
            const bool ok = p < L && f < nf;
            const float x = q.r[ok ? f * q.stride + n : 0];
            v[u] = make_float2(ok ? x : 0.f, 0.f);
        }
    } else if (q.kind == 3) {
        unsigned short w[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = t + u * BLK, f = div(p), n = p - f * (int)M;
            const bool ok = p < L && f < nf;
            w[u] = q.u[ok ? f * q.stride + n : 0];
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = t + u * BLK, f = div(p);
            v[u] = (p < L && f < nf) ? u8_sample(w[u]) : make_float2(0.f, 0.f);
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int p = t + u * BLK, f = div(p), n = p - f * (int)M;
            v[u] = (p < L && f < nf) ? frame_sample(s, M, f0 + f, n) : make_float2(0.f, 0.f);
        }
    }
}

// Gather for kernels whose frame size M and tile length L are compile-time constants (the
// power-of-two tile kernel, the compile-time mixed-radix plans).  A full workgroup (all B frames present, every one inside
// the input) reads point p = f N + n of its tile (N = M) at sample p + f (stride - N) of its first
// frame: a 32-bit byte offset off a scalar base, with no per-point bounds selects and no
// 64-bit address chain (the generic gather_tile spends ~12 VALU per point on those, and the
// live spectrum is VALU-bound).  Same samples, so the transform's results are unchanged;
// every other workgroup takes gather_tile.
template <int PER, int BLK, int N, int L>
__device__ __forceinline__ void gather_tile_ct(const FrameSrc& s, long f0, int nf, float2 (&v)[PER]) {
    constexpr int B = L / N;
    const FrameFast q = frame_fast(s, N, f0, nf);
    const int t = threadIdx.x;
    if (nf == B && (q.kind == 1 || q.kind == 3) && (B - 1) * q.stride + N < (1L << 28)) {
        const int d = (int)(q.stride - N);
        if (q.kind == 1) {
            const char* base = reinterpret_cast<const char*>(q.c);
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int p = t + u * BLK, f = p / N;
                const unsigned off = (unsigned)(p + f * d) * 8u;
                v[u] = p < L ? *reinterpret_cast<const float2*>(base + off) : make_float2(0.f, 0.f);
            }
        } else {
            const char* base = reinterpret_cast<const char*>(q.u);
            unsigned short w[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int p = t + u * BLK, f = p / N;
                const unsigned off = (unsigned)(p + f * d) * 2u;
                w[u] = p < L ? *reinterpret_cast<const unsigned short*>(base + off) : (unsigned short)0x8080;
            }
#pragma unroll
            for (int u = 0; u < PER; ++u) v[u] = u8_sample(w[u]);
        }
        return;
    }
    gather_tile<PER, BLK>(s, N, f0, nf, L, [](int p) { return p / N; }, v);
}

// Store modes (bin k of frame f):
//   0 collated fft: out[(k + M/2) mod M] = X[k] * norm (fft.rs:14-26)
//   1 rfft: collated [M/2, M) = X[0, M - M/2) * norm (fft.rs:35)
//   2 natural order, unscaled (internal: the power-of-two transforms inside Bluestein)
//   3 / 4 as 0 / 1 but the f32 magnitude in dB, 20 log10(|X * norm|) -- the spectrum plots'
//     conversion (src/plot/complexseries.rs:90-92: y.norm(), then 20 * log10)
__host__ __device__ inline long store_stride(int mode, long M) {
    return (mode == 1 || mode == 4) ? M - M / 2 : M;
}
__host__ __device__ inline long store_elem_bytes(int mode) { return mode >= 3 ? 4 : 8; }
// output pointer advanced by `frames` frames
__host__ __device__ inline float2* store_advance(float2* out, long frames, long M, int mode) {
    return reinterpret_cast<float2*>(reinterpret_cast<char*>(out) +
                                     frames * store_stride(mode, M) * store_elem_bytes(mode));
}

// 20 log10 |X| = (10 log10 2) log2(re^2 + im^2): one v_log_f32 (~1 ulp of log2, i.e. < 1e-5 dB
// across the range below) instead of the library hypotf + log10f (~40 VALU per bin; the
// 1000-point live spectrum is VALU-bound).  Where re^2 + im^2 would leave the normal f32
// range (|X| outside ~1e-18 .. 1e18, and exact zeros) the library pair is used.
__device__ __forceinline__ float db_of(float2 x, float norm) {
    const float a = x.x * norm, b = x.y * norm;
    const float m2 = a * a + b * b;
    if (m2 > 1e-36f && m2 < 1e36f) return 3.01029995663981195f * __builtin_amdgcn_logf(m2);
    return 20.0f * log10f(hypotf(a, b));
}

__device__ __forceinline__ void store_bin(float2* __restrict__ out, long f, long M, long k,
                                          float2 x, int mode, float norm) {
    if (mode == 0 || mode == 3) {
        long o = k + M / 2;
        if (o >= M) o -= M;
        if (mode == 0) out[f * M + o] = make_float2(x.x * norm, x.y * norm);
        else reinterpret_cast<float*>(out)[f * M + o] = db_of(x, norm);
    } else if (mode == 1 || mode == 4) {
        const long keep = M - M / 2;
        if (k < keep) {
            if (mode == 1) out[f * keep + k] = make_float2(x.x * norm, x.y * norm);
            else reinterpret_cast<float*>(out)[f * keep + k] = db_of(x, norm);
        }
    } else {
        out[f * M + k] = x;
    }
}

}  // namespace sdrgpu
