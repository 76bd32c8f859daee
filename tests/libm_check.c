/* Host validation of unnamed-rust-sdr_amd/csrc/libm_glibc.h against this machine's glibc:
 * sinf/cosf exhaustively over all floats with |x| < LIMIT (both signs), atan2f on N random
 * (y, x) pairs drawn from four distributions.  Exit code = 0 iff bit-exact everywhere. */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "libm_glibc.h"

typedef struct { uint32_t lo, hi; uint64_t seed; long n, mis; } job;

static void* run_trig(void* a) {
    job* j = (job*)a;
    for (uint32_t u = j->lo; u < j->hi; ++u)
        for (int sg = 0; sg < 2; ++sg) {
            float x = sdr_asfloat(u | (sg ? 0x80000000u : 0u));
            const float rs = sinf(x), rc = cosf(x);
            if (sdr_asuint(rs) != sdr_asuint(sdr_sinf(x))) j->mis++;
            if (sdr_asuint(rc) != sdr_asuint(sdr_cosf(x))) j->mis++;
            float bs, bc;
            sdr_sincosf_bf(x, &bs, &bc); /* branch-free GPU form */
            if (sdr_asuint(rs) != sdr_asuint(bs)) j->mis++;
            if (sdr_asuint(rc) != sdr_asuint(bc)) j->mis++;
            sdr_sincosf_bf2(x, &bs, &bc); /* sign-after-evaluation form (the kernel's) */
            if (sdr_asuint(rs) != sdr_asuint(bs)) j->mis++;
            if (sdr_asuint(rc) != sdr_asuint(bc)) j->mis++;
        }
    return 0;
}

static inline uint64_t xs(uint64_t* s) { uint64_t x = *s; x ^= x << 13; x ^= x >> 7; x ^= x << 17; return *s = x; }

static void* run_atan2(void* a) {
    job* j = (job*)a;
    uint64_t s = j->seed;
    for (long i = 0; i < j->n; ++i) {
        uint64_t r = xs(&s);
        float y, x;
        switch (r & 3) {
        case 0: y = sdr_asfloat((uint32_t)(r >> 8)); x = sdr_asfloat((uint32_t)(xs(&s) >> 8)); break;
        case 1: y = (float)((int32_t)(r >> 32)) / 2147483648.0f; x = (float)((int32_t)(xs(&s) >> 32)) / 2147483648.0f; break;
        case 2: y = (float)((r >> 40) & 0xffffff) / 16777216.0f * ((r & 8) ? -1e-3f : 1e-3f);
                x = (float)((int32_t)(xs(&s) >> 32)) / 2147483648.0f; break;
        default: y = (float)((int32_t)(r >> 32)) / 2147483648.0f * 4;
                 x = y * (1.0f + ((float)((int32_t)(xs(&s) >> 40)) / 8388608.0f) * 1e-3f); break;
        }
        float a1 = atan2f(y, x), a2 = sdr_atan2f(y, x), a3 = sdr_atan2f_bf(y, x);
        float a4 = sdr_atan2f_bfx(y, x);
        if (sdr_asuint(a1) != sdr_asuint(a2) && !(isnan(a1) && isnan(a2))) j->mis++;
        if (sdr_asuint(a1) != sdr_asuint(a3) && !(isnan(a1) && isnan(a3))) j->mis++;
        if (sdr_asuint(a1) != sdr_asuint(a4) && !(isnan(a1) && isnan(a4))) j->mis++;
    }
    return 0;
}

/* every pair of special / boundary values (zeros, infinities, NaN, 1, tiny / huge, the
 * |k| = 60 boundary, denormals) through the fully branch-free atan2f */
static long special_pairs(void) {
    const float v[] = {0.0f, 1.0f, 2.0f, 0.5f, 3.0f, 1e-30f, 1e30f, 1e-45f, 1.17549435e-38f,
                       3.4028235e38f, INFINITY, NAN, 0x1p60f, 0x1p61f, 0x1p-60f, 0x1p-61f,
                       0x1p25f, 0x1p-29f, 0.4375f, 0.6875f, 1.1875f, 2.4375f, 1.0000001f,
                       0.99999994f, 7.0f, 1e-7f};
    const int nv = sizeof v / sizeof v[0];
    long mis = 0;
    for (int i = 0; i < nv; ++i)
        for (int j = 0; j < nv; ++j)
            for (int s = 0; s < 4; ++s) {
                const float y = (s & 1) ? -v[i] : v[i], x = (s & 2) ? -v[j] : v[j];
                const float a1 = atan2f(y, x), a4 = sdr_atan2f_bfx(y, x);
                if (sdr_asuint(a1) != sdr_asuint(a4) && !(isnan(a1) && isnan(a4))) {
                    if (mis < 10) printf("atan2f(%a, %a): glibc %a, bfx %a\n", y, x, a1, a4);
                    mis++;
                }
            }
    return mis;
}

/* the atanf tails the branch-free form leaves to its common path: |y / x| above 2^25 (and
 * past the |k| > 60 cut) and below 2^-29, every sign, 2^22 mantissa pairs per exponent step */
static long ratio_tails(void) {
    long mis = 0;
    uint64_t r = 0x243F6A8885A308D3ull;
    for (int e = -100; e <= 100; ++e) {
        if (e > -29 && e < 25) continue;
        for (int i = 0; i < (1 << 14); ++i) {
            r = r * 6364136223846793005ull + 1442695040888963407ull;
            const float my = 1.0f + (float)((r >> 40) & 0x7fffff) * 0x1p-23f;
            const float mx = 1.0f + (float)((r >> 17) & 0x7fffff) * 0x1p-23f;
            const float y0 = ldexpf(my, e / 2 + (e & 1)), x0 = ldexpf(mx, -(e / 2));
            for (int s = 0; s < 4; ++s) {
                const float y = (s & 1) ? -y0 : y0, x = (s & 2) ? -x0 : x0;
                const float a1 = atan2f(y, x), a4 = sdr_atan2f_bfx(y, x);
                if (sdr_asuint(a1) != sdr_asuint(a4) && !(isnan(a1) && isnan(a4))) {
                    if (mis < 10) printf("atan2f(%a, %a): glibc %a, bfx %a\n", y, x, a1, a4);
                    mis++;
                }
            }
        }
    }
    return mis;
}

int main(int argc, char** argv) {
    float limit = argc > 1 ? (float)atof(argv[1]) : 120.0f;
    long npairs = argc > 2 ? atol(argv[2]) : 100000000L;
    const int T = 8;
    pthread_t th[8];
    job jb[8];
    uint32_t top = sdr_asuint(limit);
    long mt = 0, ma = 0;
    for (int t = 0; t < T; ++t) {
        jb[t].lo = (uint32_t)((uint64_t)top * t / T); jb[t].hi = (uint32_t)((uint64_t)top * (t + 1) / T);
        jb[t].mis = 0; pthread_create(&th[t], 0, run_trig, &jb[t]);
    }
    for (int t = 0; t < T; ++t) { pthread_join(th[t], 0); mt += jb[t].mis; }
    for (int t = 0; t < T; ++t) {
        jb[t].seed = 0x9E3779B97F4A7C15ull * (t + 1); jb[t].n = npairs / T; jb[t].mis = 0;
        pthread_create(&th[t], 0, run_atan2, &jb[t]);
    }
    for (int t = 0; t < T; ++t) { pthread_join(th[t], 0); ma += jb[t].mis; }
    const long ms = special_pairs() + ratio_tails();
    printf("sinf/cosf |x|<%g: %ld mismatches; atan2f %ld pairs: %ld mismatches; special pairs: %ld\n",
           limit, mt, npairs, ma, ms);
    return (mt || ma || ms) ? 1 : 0;
}
