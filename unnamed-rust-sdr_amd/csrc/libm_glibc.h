/*
 * libm_glibc.h -- bit-exact restatements of the glibc 2.35 (x86-64) sinf, cosf and atan2f
 * that the reference calls through Rust std (f32::sin/cos -> sinf/cosf, Complex::arg ->
 * f32::atan2 -> atan2f; reference src/filter/pll.rs:72,76).
 *
 * Why: the reference PLL (pll.rs:70-85) is a chaotic recurrence on noisy input -- a 1-ulp
 * difference in any sample's sin/cos/atan2 shifts the next cycle slip and the outputs
 * diverge (measured: FMA vs no-FMA builds of the same restatement differ by 3 % L2).  The
 * only way to reproduce the reference's outputs is to reproduce its libm bit for bit.
 *
 *  - sinf/cosf: glibc sysdeps/ieee754/flt-32 s_sinf.c / s_cosf.c with sincosf.h (double
 *    evaluation, single-step range reduction for |x| < 120), table __sincosf_table read
 *    from the system libm binary.  x86-64 glibc dispatches to an FMA build on CPUs with
 *    FMA (every `a + b*c` contracted); SDR_LIBM_FMA selects that variant.
 *  - atan2f: fdlibm-derived e_atan2f.c / s_atanf.c (pure f32, not contracted on x86-64).
 *
 * The file compiles as C (gcc, for the host validation in tests/) and as HIP device code
 * (hipcc).  Explicit fma()/fmaf() only where the original contracts; everything else must
 * be compiled with contraction OFF (-ffp-contract=off).  Validated exhaustively over
 * |x| < 120 (sinf/cosf) and on random/targeted inputs (atan2f) by
 * tests/test_libm_restatement.py.
 */
#ifndef SDR_LIBM_GLIBC_H
#define SDR_LIBM_GLIBC_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#define SDR_LIBM_FN __host__ __device__ static inline
#else
#include <math.h>
#define SDR_LIBM_FN static inline
#endif

#ifndef SDR_LIBM_FMA
#define SDR_LIBM_FMA 1
#endif

#if SDR_LIBM_FMA
#define SDR_MAD(a, b, c) fma((a), (b), (c)) /* c + a*b, contracted */
#else
#define SDR_MAD(a, b, c) ((c) + (a) * (b))
#endif

SDR_LIBM_FN uint32_t sdr_asuint(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
SDR_LIBM_FN float sdr_asfloat(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* __sincosf_table[2] (glibc sysdeps/ieee754/flt-32/sincosf_data.c), field order
 * sign[4], hpi_inv (2/pi * 2^24), hpi, c0, c1, s1, c2, s2, c3, s3, c4. */
#define SDR_HPI_INV 0x1.45f306dc9c883p+23
#define SDR_HPI 0x1.921fb54442d18p+0
#define SDR_C1 -0x1.ffffffd0c621cp-2
#define SDR_S1 -0x1.555545995a603p-3
#define SDR_C2 0x1.55553e1068f19p-5
#define SDR_S2 0x1.1107605230bc4p-7
#define SDR_C3 -0x1.6c087e89a359dp-10
#define SDR_S3 -0x1.994eb3774cf24p-13
#define SDR_C4 0x1.99343027bf8c3p-16

SDR_LIBM_FN uint32_t sdr_abstop12(float x) { return (sdr_asuint(x) >> 20) & 0x7ff; }

/* sinf_poly (sincosf.h): n even -> sine polynomial, odd -> cosine polynomial; neg selects
 * table[1] (cosine coefficients negated). */
SDR_LIBM_FN float sdr_sinf_poly(double x, double x2, int n, int neg) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = SDR_MAD(x2, SDR_S3, SDR_S2);
        double x7 = x3 * x2;
        double s = SDR_MAD(x3, SDR_S1, x);
        return (float)SDR_MAD(x7, s1, s);
    } else {
        const double c0 = neg ? -1.0 : 1.0;
        const double kc1 = neg ? -SDR_C1 : SDR_C1, kc2 = neg ? -SDR_C2 : SDR_C2;
        const double kc3 = neg ? -SDR_C3 : SDR_C3, kc4 = neg ? -SDR_C4 : SDR_C4;
        double x4 = x2 * x2;
        double c2 = SDR_MAD(x2, kc4, kc3);
        double c1 = SDR_MAD(x2, kc1, c0);
        double x6 = x4 * x2;
        double c = SDR_MAD(x4, kc2, c1);
        return (float)SDR_MAD(x6, c2, c);
    }
}

/* reduce_fast, !TOINT_INTRINSICS form (x86-64): quadrant in bits 24..31 of r. */
SDR_LIBM_FN double sdr_reduce_fast(double x, int* np) {
    double r = x * SDR_HPI_INV;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
#if SDR_LIBM_FMA
    return fma(-(double)n, SDR_HPI, x);
#else
    return x - n * SDR_HPI;
#endif
}

/* sinf for |y| < 120 (the PLL phase is 2 pi * fract(.) so |y| < 2 pi). */
SDR_LIBM_FN float sdr_sinf(float y) {
    double x = y;
    if (sdr_abstop12(y) < 0x3f4 /* abstop12(pio4f) */) {
        double s = x * x;
        if (sdr_abstop12(y) < 0x398 /* abstop12(0x1p-12f) */) return y;
        return sdr_sinf_poly(x, s, 0, 0);
    }
    int n;
    x = sdr_reduce_fast(x, &n);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0; /* sign[n & 3] */
    return sdr_sinf_poly(x * s, x * x, n, (n & 2) != 0);
}

SDR_LIBM_FN float sdr_cosf(float y) {
    double x = y;
    if (sdr_abstop12(y) < 0x3f4) {
        double x2 = x * x;
        if (sdr_abstop12(y) < 0x398) return 1.0f;
        return sdr_sinf_poly(x, x2, 1, 0);
    }
    int n;
    x = sdr_reduce_fast(x, &n);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sdr_sinf_poly(x * s, x * x, n ^ 1, (n & 2) != 0);
}

/* ---- fdlibm atanf (glibc sysdeps/ieee754/flt-32/s_atanf.c) ---- */
SDR_LIBM_FN float sdr_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f,
                             1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f,
                             7.5497894159e-08f};
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const float one = 1.0f, huge = 1.0e30f;
    float w, s1, s2, z;
    int32_t ix, hx, id;
    hx = (int32_t)sdr_asuint(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) { /* |x| >= 2^25 */
        if (ix > 0x7f800000) return x + x; /* NaN */
        if (hx > 0) return atanhi[3] + atanlo[3];
        return -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) { /* |x| < 0.4375 */
        if (ix < 0x31000000) { /* |x| < 2^-29 */
            if (huge + x > one) return x;
        }
        id = -1;
    } else {
        x = sdr_asfloat(sdr_asuint(x) & 0x7fffffffu); /* fabsf */
        if (ix < 0x3f980000) {       /* |x| < 1.1875 */
            if (ix < 0x3f300000) {   /* 7/16 <= |x| < 11/16 */
                id = 0;
                x = ((float)2.0 * x - one) / ((float)2.0 + x);
            } else { /* 11/16 <= |x| < 19/16 */
                id = 1;
                x = (x - one) / (x + one);
            }
        } else {
            if (ix < 0x401c0000) { /* |x| < 2.4375 */
                id = 2;
                x = (x - (float)1.5) / (one + (float)1.5 * x);
            } else { /* 2.4375 <= |x| < 2^66 */
                id = 3;
                x = -(float)1.0 / x;
            }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -z : z;
}

/* ---- fdlibm atan2f (glibc sysdeps/ieee754/flt-32/e_atan2f.c) ---- */
SDR_LIBM_FN float sdr_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, zero = 0.0f;
    const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f;
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    float z;
    int32_t k, m, hx, hy, ix, iy;
    hx = (int32_t)sdr_asuint(x);
    ix = hx & 0x7fffffff;
    hy = (int32_t)sdr_asuint(y);
    iy = hy & 0x7fffffff;
    if ((ix > 0x7f800000) || (iy > 0x7f800000)) return x + y; /* NaN */
    if (hx == 0x3f800000) return sdr_atanf(y);                 /* x = 1.0 */
    m = ((hy >> 31) & 1) | ((hx >> 30) & 2);                   /* 2*sign(x)+sign(y) */
    if (iy == 0) {
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return (float)3.0 * pi_o_4 + tiny;
            default: return (float)-3.0 * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
            case 0: return zero;
            case 1: return -zero;
            case 2: return pi + tiny;
            default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    k = (iy - ix) >> 23;
    if (k > 60) z = pi_o_2 + (float)0.5 * pi_lo; /* |y/x| > 2^60 */
    else if (hx < 0 && k < -60) z = 0.0f;        /* |y|/x < -2^60 */
    else {
        const float q = y / x;
        z = sdr_atanf(sdr_asfloat(sdr_asuint(q) & 0x7fffffffu));
    }
    switch (m) {
    case 0: return z;
    case 1: return sdr_asfloat(sdr_asuint(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}


/* ---------------------------------------------------------------------------------------
 * Branch-free forms for SIMD execution (a wave runs every taken path of a divergent
 * branch).  Same per-lane arithmetic as the functions above -- only control flow differs:
 *  - sincos: for |y| < 0.75 glibc skips reduce_fast, but there reduce_fast yields n = 0 and
 *    x - 0*hpi == x exactly, so always reducing is bit-identical; one reduction feeds both
 *    the sine and the cosine polynomial, and the quadrant picks which is sin and which cos.
 *  - atanf: the five argument-reduction cases become selects of one numerator / one
 *    denominator (each formed with the original operation order), then ONE division.
 *  - atan2f: the sign quadrant switch becomes selects; true special cases (zero, inf, nan,
 *    |y/x| beyond 2^+-60, x == 1) fall back to the reference function.
 * Validated bit-exact against the host libm by tests/test_libm_restatement.py.
 * ------------------------------------------------------------------------------------- */
/* As sdr_sincosf_bf with fewer instructions: both polynomials are odd/even in a way that
 * makes the sign handling exact AFTER evaluation -- sin_poly(-x) = -sin_poly(x) and the
 * negated-coefficient cosine table gives exactly -cos_poly (every fma / mul / add of the
 * evaluation commutes with negation under round-to-nearest) -- so one positive-coefficient
 * evaluation of each and a sign flip of the f32 results replace the f64 selects. */
SDR_LIBM_FN void sdr_sincosf_bf2(float y, float* sinp, float* cosp) {
    int n;
    const double xr = sdr_reduce_fast((double)y, &n);
    const double x2 = xr * xr;
    const double x3 = xr * x2;
    const double s1 = SDR_MAD(x2, SDR_S3, SDR_S2);
    const double x7 = x3 * x2;
    const double ss = SDR_MAD(x3, SDR_S1, xr);
    const float sp0 = (float)SDR_MAD(x7, s1, ss);         /* sin_poly(xr) */
    const double x4 = x2 * x2;
    const double c2 = SDR_MAD(x2, SDR_C4, SDR_C3);
    const double c1 = SDR_MAD(x2, SDR_C1, 1.0);
    const double x6 = x4 * x2;
    const double cc = SDR_MAD(x4, SDR_C2, c1);
    const float cp0 = (float)SDR_MAD(x6, c2, cc);         /* cos_poly(xr), table[0] */
    /* sign[n & 3] of sinf (negative for n & 3 in {1, 2}, i.e. bit 1 of n + 1) and of the
     * cosine polynomial (n & 2), as bit arithmetic rather than compares and selects */
    const uint32_t sgn_s = ((uint32_t)(n + 1) & 2u) << 30;
    const uint32_t sgn_c = ((uint32_t)n & 2u) << 30;
    const float sp = sdr_asfloat(sdr_asuint(sp0) ^ sgn_s);
    const float cp = sdr_asfloat(sdr_asuint(cp0) ^ sgn_c);
    /* glibc returns y / 1.0f for |y| < 2^-12 without the polynomial; here the polynomial's
     * own result is used: n = 0, xr = y, and sin_poly(y) = y (1 - e) with e < 2^-26, cos_poly
     * = 1 - y^2/2 > 1 - 2^-25, which round to exactly y and 1.0f -- except sin(-0), where
     * x7 * s1 = +0 turns the sum into +0: zeros keep their own sign (checked exhaustively
     * with the rest, tests/libm_check.c) */
    *sinp = (y == 0.0f) ? y : ((n & 1) ? cp : sp);
    *cosp = (n & 1) ? sp : cp;
}

SDR_LIBM_FN void sdr_sincosf_bf(float y, float* sinp, float* cosp) {
    int n;
    const double xr = sdr_reduce_fast((double)y, &n);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    const int neg = (n & 2) != 0;
    const double xs = xr * s, x2 = xr * xr;
    /* sine polynomial of xs (n even branch of sinf_poly) */
    const double x3 = xs * x2;
    const double s1 = SDR_MAD(x2, SDR_S3, SDR_S2);
    const double x7 = x3 * x2;
    const double ss = SDR_MAD(x3, SDR_S1, xs);
    const float sp = (float)SDR_MAD(x7, s1, ss);
    /* cosine polynomial (n odd branch), table[neg] */
    const double c0 = neg ? -1.0 : 1.0;
    const double kc1 = neg ? -SDR_C1 : SDR_C1, kc2 = neg ? -SDR_C2 : SDR_C2;
    const double kc3 = neg ? -SDR_C3 : SDR_C3, kc4 = neg ? -SDR_C4 : SDR_C4;
    const double x4 = x2 * x2;
    const double c2 = SDR_MAD(x2, kc4, kc3);
    const double c1 = SDR_MAD(x2, kc1, c0);
    const double x6 = x4 * x2;
    const double cc = SDR_MAD(x4, kc2, c1);
    const float cp = (float)SDR_MAD(x6, c2, cc);
    const int tiny = sdr_abstop12(y) < 0x398; /* |y| < 2^-12: sinf returns y, cosf 1 */
    *sinp = tiny ? y : ((n & 1) ? cp : sp);
    *cosp = tiny ? 1.0f : ((n & 1) ? sp : cp);
}

/* f32 division a / b, correctly rounded, for finite nonzero a, b whose quotient is a normal
 * float -- the only operands whose quotient the branch-free atan2f/atanf below use (zeros,
 * infinities, NaNs and |y/x| beyond 2^+-60 are replaced by the special-case selects).  On the
 * device it is evaluated in f64: a reciprocal refined once by Newton and a corrected quotient
 * (relative error < 2^-52), rounded once to f32.  The exact quotient of two 24-bit significands
 * is never within 2^-49 (relative) of an f32 rounding midpoint, so that rounding equals
 * IEEE a / b; checked bit-exact against the compiler's a / b on 2^36 GPU pairs
 * (tools/fdiv_check.hip).  Seven dependent f64 ops instead of the ten-deep v_div_scale /
 * v_rcp / fma / v_div_fmas / v_div_fixup chain with its VCC hazards. */
SDR_LIBM_FN float sdr_fdiv(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double bd = (double)b, ad = (double)a;
    const double r0 = __builtin_amdgcn_rcp(bd);
    const double r1 = fma(r0, fma(-bd, r0, 1.0), r0);
    const double q0 = ad * r1;
    return (float)fma(fma(-bd, q0, ad), r1, q0);
#else
    return a / b;
#endif
}

/* f32 division num / den restricted to atanf's argument reduction below: den in [1.6, 2^25),
 * num in [-1, 2) and a normal or exactly zero quotient (lanes outside that -- |x| >= 2^25 or
 * the small case -- discard the quotient through the selects that follow).  There the division needs no operand
 * scaling, so on the device it is the f32 reciprocal, one Newton step and two corrected
 * quotients -- the IEEE sequence the compiler emits around v_div_scale / v_div_fmas /
 * v_div_fixup, without those three.  Eight full-rate f32 ops instead of sdr_fdiv's half-rate
 * f64 chain; checked bit-exact against IEEE num / den inside sdr_atanf_bf for every
 * non-negative finite float argument (tools/atanf_check.hip, 2^31 - 2^23 inputs). */
SDR_LIBM_FN float sdr_fdiv_n(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float y1 = fmaf(fmaf(-b, y0, 1.0f), y0, y0);
    const float q0 = a * y1;
    const float q1 = fmaf(fmaf(-b, q0, a), y1, q0);
    return fmaf(fmaf(-b, q1, a), y1, q1);
#else
    return a / b;
#endif
}

/* ieee_div != 0: the reduction divides with the IEEE operator (the check tool's ground truth) */
SDR_LIBM_FN float sdr_atanf_core(float x, int ieee_div) {
    /* finite x (sdr_atan2f_bf routes NaN through the reference function) */
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
                atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
                atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const float one = 1.0f;
    const int32_t hx = (int32_t)sdr_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    const float ax = sdr_asfloat((uint32_t)ix);
    /* reduction case (s_atanf.c): |x| < 0.4375 small; else the first of c0 (< 11/16),
     * c1 (< 19/16), c2 (< 39/16) that holds, or none (id 3) */
    const int small = ix < 0x3ee00000;
    const int c0 = ix < 0x3f300000, c1 = ix < 0x3f980000, c2 = ix < 0x401c0000;
    const float num0 = (float)2.0 * ax - one, den0 = (float)2.0 + ax;
    const float num1 = ax - one, den1 = ax + one;
    const float num2 = ax - (float)1.5, den2 = one + (float)1.5 * ax;
    const float num = c0 ? num0 : c1 ? num1 : c2 ? num2 : -(float)1.0;
    const float den = c0 ? den0 : c1 ? den1 : c2 ? den2 : ax;
    const float q = ieee_div ? num / den : sdr_fdiv_n(num, den);
    const float xr = small ? x : q;
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const float hi = c0 ? atanhi0 : c1 ? atanhi1 : c2 ? atanhi2 : atanhi3;
    const float lo = c0 ? atanlo0 : c1 ? atanlo1 : c2 ? atanlo2 : atanlo3;
    const float rsmall = xr - xr * (s1 + s2);
    const float zz = hi - ((xr * (s1 + s2) - lo) - xr);
    const float rbig = (hx < 0) ? -zz : zz;
    /* |x| >= 2^25: +-(atanhi[3] + atanlo[3]); |x| < 2^-29: x itself (s_atanf.c) */
    const float rhuge = (hx > 0) ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
    float rc = small ? rsmall : rbig;
#if defined(__HIP_DEVICE_COMPILE__)
    /* opaque: keeps the compiler from turning the |x| >= 2^25 select below into an exec-mask
     * branch around the whole evaluation (370 vs 396 ns per PLL sample-chain) */
    __asm__ volatile("" : "+v"(rc));
#endif
    /* s_atanf.c returns x itself for |x| < 2^-29: the small-case polynomial gives exactly x
     * there (x (s1 + s2) < 2^-58 |x|), so no select (atan2f's argument is |y / x| >= +0) */
    return ix >= 0x4c000000 ? rhuge : rc;
}

SDR_LIBM_FN float sdr_atanf_bf(float x) { return sdr_atanf_core(x, 0); }

SDR_LIBM_FN float sdr_atan2f_bf(float y, float x) {
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)sdr_asuint(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)sdr_asuint(y), iy = hy & 0x7fffffff;
    const int32_t k = (iy - ix) >> 23;
    /* common case: both finite and nonzero, x != 1, |k| <= 60 */
    const int special = (ix >= 0x7f800000) | (iy >= 0x7f800000) | (ix == 0) | (iy == 0) |
                        (hx == 0x3f800000) | (k > 60) | (k < -60);
    if (special) return sdr_atan2f(y, x);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const float qq = y / x;
    const float z = sdr_atanf_bf(sdr_asfloat(sdr_asuint(qq) & 0x7fffffffu));
    const float t = z - pi_lo;
    const float r2 = pi - t, r3 = t - pi;
    const float r1 = sdr_asfloat(sdr_asuint(z) ^ 0x80000000u);
    return m == 0 ? z : m == 1 ? r1 : m == 2 ? r2 : r3;
}

/* Fully branch-free atan2f: the reference's special cases (e_atan2f.c) as selects of
 * constants instead of a fallback call, so a wave never runs -- or carries the code of -- the
 * reference function.  Order of the reference's checks: NaN; x == 1 (atanf(y): the common
 * path gives the same bits, atanf being exactly odd in fdlibm); y == 0; x == 0; x = inf;
 * y = inf; |y/x| beyond 2^60 (z = pi/2 + pi_lo/2) or below 2^-60 with x < 0 (z = 0); else
 * z = atanf(|y/x|); then the quadrant from the signs. */
SDR_LIBM_FN float sdr_atan2f_bfx(float y, float x) {
    const float tiny = 1.0e-30f, zero = 0.0f;
    const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f;
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)sdr_asuint(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)sdr_asuint(y), iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    /* common path (its value is discarded wherever a special case applies) */
    const float qq = sdr_fdiv(y, x);
    const float za = sdr_atanf_bf(sdr_asfloat(sdr_asuint(qq) & 0x7fffffffu));
    /* k = (iy - ix) >> 23 > 60 (|y / x| > 2^60): e_atan2f.c's pi_o_2 + 0.5 pi_lo rounds to the same float as
     * atanf's |x| >= 2^25 constant atanhi[3] + atanlo[3], which the common path returns */
    /* quadrant (e_atan2f.c's switch on m): x < 0 gives pi - (z - pi_lo), x >= 0 gives z, and
     * y's sign is copied on -- m == 1's -z and m == 3's (z - pi_lo) - pi are exactly the
     * negations (round-to-nearest is symmetric, neither is zero, z >= +0).  The reference's
     * z = 0 for x < 0 and |y / x| < 2^-60 needs no select either: there za < 2^-59 is below
     * half an ulp of pi_lo (2^-48), so za - pi_lo rounds to exactly 0 - pi_lo. */
    const float zq = (hx < 0) ? pi - (za - pi_lo) : za;
    const float gen = sdr_asfloat((sdr_asuint(zq) & 0x7fffffffu) | ((uint32_t)hy & 0x80000000u));
    /* special cases, reference order (later checks apply only where earlier ones did not) */
    const float by_m_pi = (m <= 1) ? y : (m == 2 ? pi + tiny : -pi - tiny);          /* y == 0 */
    const float half = (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;                  /* x == 0, y = inf */
    const float infinf = m == 0 ? pi_o_4 + tiny : m == 1 ? -pi_o_4 - tiny
                       : m == 2 ? (float)3.0 * pi_o_4 + tiny : (float)-3.0 * pi_o_4 - tiny;
    const float inffin = m == 0 ? zero : m == 1 ? -zero : m == 2 ? pi + tiny : -pi - tiny;
    float r = gen;
#if defined(__HIP_DEVICE_COMPILE__)
    /* a wave skips the special-case selects when none of its lanes needs them */
    /* NaN, +-inf or +-0 in either operand: one class test each (mask 0x267) */
    const int spec = __builtin_amdgcn_classf(x, 0x267) | __builtin_amdgcn_classf(y, 0x267);
    if (!__builtin_amdgcn_ballot_w64(spec)) return r;
#endif
    r = (iy == 0x7f800000) ? half : r;
    r = (ix == 0x7f800000) ? ((iy == 0x7f800000) ? infinf : inffin) : r;
    r = (ix == 0) ? half : r;
    r = (iy == 0) ? by_m_pi : r;
    r = ((ix > 0x7f800000) | (iy > 0x7f800000)) ? x + y : r;
    return r;
}

#endif /* SDR_LIBM_GLIBC_H */
