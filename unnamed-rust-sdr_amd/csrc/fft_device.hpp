// fft_device.hpp -- register-level radix-2/4/8/16 DFT butterflies and complex helpers
// shared by the overlap-save FIR and the Stockham FFT kernels (gfx950).
#pragma once

#include "common.hpp"

namespace sdrgpu {
namespace fftd {

// Native 2-wide vector view of a complex value: one VGPR pair, so complex adds are single
// v_pk_add_f32 and the +-i rotations below fold into that instruction's op_sel / neg bits
// (the compiler does not form those from float2 struct code and emits swaps instead).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v vv(float2 a) { return __builtin_bit_cast(f2v, a); }
__device__ __forceinline__ float2 ff(f2v a) { return __builtin_bit_cast(float2, a); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return ff(vv(a) + vv(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return ff(vv(a) - vv(b)); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }

// a + (-i) b = (a.x + b.y, a.y - b.x): one v_pk_add_f32 (src1 halves swapped, hi negated)
__device__ __forceinline__ f2v add_mi(f2v a, f2v b) {
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// a - (-i) b = a + i b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ f2v sub_mi(f2v a, f2v b) {
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
    const f2v z = {0.f, 0.f};
    return ff(INV ? sub_mi(z, vv(a)) : add_mi(z, vv(a)));
}

// a * W16^m (forward sign) or a * conj(W16^m) (inverse); m = 0..15
template <bool INV>
__device__ __forceinline__ float2 twm(float2 a, int m16) {
    constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f;
    constexpr float c2 = 0.70710678118654752f;
    const f2v x = vv(a);
    const f2v z = {0.f, 0.f};
    switch (m16 & 15) {
    case 0: return a;
    case 2: return ff((INV ? sub_mi(x, x) : add_mi(x, x)) * c2);      // (1 -+ i)/sqrt2
    case 4: return ff(INV ? sub_mi(z, x) : add_mi(z, x));              // -+i
    case 6: return ff((INV ? add_mi(x, x) : sub_mi(x, x)) * (-c2));   // (-1 -+ i)/sqrt2
    case 8: return ff(-x);
    case 10: return ff((INV ? sub_mi(x, x) : add_mi(x, x)) * (-c2));  // (-1 +- i)/sqrt2
    case 12: return ff(INV ? add_mi(z, x) : sub_mi(z, x));             // +-i
    case 14: return ff((INV ? add_mi(x, x) : sub_mi(x, x)) * c2);     // (1 +- i)/sqrt2
    default: break;
    }
    // generic: the W16 table value (conjugated for the inverse)
    float2 w;
    switch (m16 & 15) {
    case 1: w = make_float2(c1, -s1); break;
    case 3: w = make_float2(s1, -c1); break;
    case 5: w = make_float2(-s1, -c1); break;
    case 7: w = make_float2(-c1, -s1); break;
    case 9: w = make_float2(-c1, s1); break;
    case 11: w = make_float2(-s1, c1); break;
    case 13: w = make_float2(s1, c1); break;
    default: w = make_float2(c1, s1); break;
    }
    if (INV) w.y = -w.y;
    return cmul(a, w);
}

template <bool INV>
__device__ __forceinline__ void dft2(float2& a, float2& b) {
    const f2v t = vv(a), u = vv(b);
    a = ff(t + u);
    b = ff(t - u);
}

// in-place 4-point DFT, natural-order output: 8 v_pk_add_f32
template <bool INV>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const f2v x0 = vv(a0), x1 = vv(a1), x2 = vv(a2), x3 = vv(a3);
    const f2v s02 = x0 + x2, d02 = x0 - x2, s13 = x1 + x3, d13 = x1 - x3;
    a0 = ff(s02 + s13);
    a2 = ff(s02 - s13);
    a1 = ff(INV ? sub_mi(d02, d13) : add_mi(d02, d13));
    a3 = ff(INV ? add_mi(d02, d13) : sub_mi(d02, d13));
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
