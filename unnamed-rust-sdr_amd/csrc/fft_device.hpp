// fft_device.hpp -- register-level radix-2/4/8/16 DFT butterflies and complex helpers
// shared by the overlap-save FIR and the Stockham FFT kernels (gfx950).
#pragma once

#include "common.hpp"

namespace sdrgpu {
namespace fftd {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

// exp(-+2 pi i m / 16) for m = 0..15 (sign applied by caller via INV)
__device__ __forceinline__ float2 w16(int m) {
    constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f;
    constexpr float c2 = 0.70710678118654752f;
    switch (m & 15) {
    case 0: return make_float2(1.f, 0.f);
    case 1: return make_float2(c1, -s1);
    case 2: return make_float2(c2, -c2);
    case 3: return make_float2(s1, -c1);
    case 4: return make_float2(0.f, -1.f);
    case 5: return make_float2(-s1, -c1);
    case 6: return make_float2(-c2, -c2);
    case 7: return make_float2(-c1, -s1);
    case 8: return make_float2(-1.f, 0.f);
    case 9: return make_float2(-c1, s1);
    case 10: return make_float2(-c2, c2);
    case 11: return make_float2(-s1, c1);
    case 12: return make_float2(0.f, 1.f);
    case 13: return make_float2(s1, c1);
    case 14: return make_float2(c2, c2);
    default: return make_float2(c1, s1);
    }
}

template <bool INV>
__device__ __forceinline__ float2 twm(float2 a, int m16) {
    // a * W16^m (forward sign) or a * conj(W16^m) (inverse)
    float2 w = w16(m16);
    if (INV) w.y = -w.y;
    return cmul(a, w);
}

template <bool INV>
__device__ __forceinline__ void dft2(float2& a, float2& b) {
    float2 t = a;
    a = cadd(t, b);
    b = csub(t, b);
}

// in-place 4-point DFT, natural-order output
template <bool INV>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    float2 s02 = cadd(a0, a2), d02 = csub(a0, a2);
    float2 s13 = cadd(a1, a3), d13 = mul_mi<INV>(csub(a1, a3));
    a0 = cadd(s02, s13);
    a2 = csub(s02, s13);
    a1 = cadd(d02, d13);
    a3 = csub(d02, d13);
}

// generic R = R1*R2 split: n = R2*n1 + n2 ; k = k1 + R1*k2
//   a[n2][k1] = DFT_R1 over n1 of v[R2*n1+n2];  a *= W_R^(n2*k1);  X[k1+R1*k2] = DFT_R2 over n2
template <int R, bool INV> struct Dft;

template <bool INV> struct Dft<2, INV> {
    __device__ __forceinline__ static void run(float2* v) { dft2<INV>(v[0], v[1]); }
};
template <bool INV> struct Dft<4, INV> {
    __device__ __forceinline__ static void run(float2* v) { dft4<INV>(v[0], v[1], v[2], v[3]); }
};
template <bool INV> struct Dft<8, INV> {
    // n = 2*n1 + n2 (n1<4, n2<2); k = k1 + 4*k2
    __device__ __forceinline__ static void run(float2* v) {
        float2 a[2][4];
#pragma unroll
        for (int n2 = 0; n2 < 2; ++n2) {
            float2 t[4];
#pragma unroll
            for (int n1 = 0; n1 < 4; ++n1) t[n1] = v[2 * n1 + n2];
            dft4<INV>(t[0], t[1], t[2], t[3]);
#pragma unroll
            for (int k1 = 0; k1 < 4; ++k1) a[n2][k1] = (n2 * k1) ? twm<INV>(t[k1], 2 * n2 * k1) : t[k1];
        }
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            float2 p = a[0][k1], q = a[1][k1];
            dft2<INV>(p, q);
            v[k1] = p;
            v[k1 + 4] = q;
        }
    }
};
template <bool INV> struct Dft<16, INV> {
    // n = 4*n1 + n2 (n1,n2<4); k = k1 + 4*k2
    __device__ __forceinline__ static void run(float2* v) {
        float2 a[4][4];
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) {
            float2 t0 = v[n2], t1 = v[4 + n2], t2 = v[8 + n2], t3 = v[12 + n2];
            dft4<INV>(t0, t1, t2, t3);
            a[n2][0] = t0;
            a[n2][1] = n2 ? twm<INV>(t1, n2) : t1;
            a[n2][2] = n2 ? twm<INV>(t2, 2 * n2) : t2;
            a[n2][3] = n2 ? twm<INV>(t3, 3 * n2) : t3;
        }
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            float2 t0 = a[0][k1], t1 = a[1][k1], t2 = a[2][k1], t3 = a[3][k1];
            dft4<INV>(t0, t1, t2, t3);
            v[k1] = t0;
            v[k1 + 4] = t1;
            v[k1 + 8] = t2;
            v[k1 + 12] = t3;
        }
    }
};

// v[r] *= w^r for r = 1..R-1 with a log-depth power tree (w^2 = w*w, w^3 = w^2*w,
// w^4 = w^2*w^2, ...): at most log2(R) dependent complex multiplies instead of R-2.
template <int R>
__device__ __forceinline__ void twiddle_tree(float2* v, float2 w) {
    float2 p[R];
    p[1] = w;
#pragma unroll
    for (int r = 2; r < R; ++r) {
        const int a = (r & (r - 1)) ? (r & (r - 1)) : r / 2;  // r with its lowest set bit cleared, or r/2
        p[r] = cmul(p[a], p[r - a]);
    }
#pragma unroll
    for (int r = 1; r < R; ++r) v[r] = cmul(v[r], p[r]);
}

// v[r] *= w^r, r = 1..R-1, with w = tw[m] (forward table) conjugated for the inverse.
template <int R, bool INV>
__device__ __forceinline__ void twiddle(float2* v, const float2* __restrict__ tw, int m) {
    float2 w = tw[m];
    if (INV) w.y = -w.y;
    twiddle_tree<R>(v, w);
}

}  // namespace fftd
}  // namespace sdrgpu
