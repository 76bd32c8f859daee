/*
 * oracle.c -- CPU restatement of the agrif/unnamed-rust-sdr hot path (TEST ONLY).
 * See oracle.h for the contract.  Build: oracle/Makefile (-O2 -ffp-contract=off).
 * Every function cites the reference file:line it restates.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__FLT_EVAL_METHOD__) && __FLT_EVAL_METHOD__ != 0
#error "f32 arithmetic must evaluate in f32 (x86-64 SSE), as Rust does"
#endif

typedef struct { float re, im; } c32;

/* num-complex 0.2 arithmetic, as used by Convolve::accumulate (convolve.rs:13-15):
 *   Complex * f32      = (re*c, im*c)
 *   Complex * Complex  = (a.re*b.re - a.im*b.im, a.re*b.im + a.im*b.re)
 *   AddAssign          = component-wise += */
static inline c32 cmul_r(c32 a, float c) { c32 r = {a.re * c, a.im * c}; return r; }
static inline c32 cmul(c32 a, c32 b) {
    c32 r;
    r.re = a.re * b.re - a.im * b.im;
    r.im = a.re * b.im + a.im * b.re;
    return r;
}

/* ================================ FIR ================================= */
struct oracle_fir {
    int sk, tk;            /* sample / tap kind */
    size_t K;
    uint32_t D;
    float* taps;           /* K (f32) or 2K (c64) */
    float* ring;           /* 2K samples (doubled ring, newest at [head]) */
    size_t head;
    uint64_t seen;         /* samples consumed (decimation phase) */
};

oracle_fir* oracle_fir_create(int sk, int tk, const float* taps, size_t ntaps,
                              uint32_t decim) {
    if (ntaps == 0 || decim == 0) return NULL;
    if (sk == ORACLE_F32 && tk == ORACLE_C64) return NULL; /* f32: !Mul<Complex> */
    oracle_fir* f = (oracle_fir*)calloc(1, sizeof(*f));
    f->sk = sk; f->tk = tk; f->K = ntaps; f->D = decim;
    size_t tw = (tk == ORACLE_C64) ? 2 : 1, sw = (sk == ORACLE_C64) ? 2 : 1;
    f->taps = (float*)malloc(sizeof(float) * tw * ntaps);
    memcpy(f->taps, taps, sizeof(float) * tw * ntaps);
    f->ring = (float*)calloc(2 * ntaps * sw, sizeof(float));
    oracle_fir_reset(f);
    return f;
}

void oracle_fir_destroy(oracle_fir* f) {
    if (!f) return;
    free(f->taps); free(f->ring); free(f);
}

/* Fir::new zero-fills the history (fir.rs:12-19). */
void oracle_fir_reset(oracle_fir* f) {
    size_t sw = (f->sk == ORACLE_C64) ? 2 : 1;
    memset(f->ring, 0, sizeof(float) * 2 * f->K * sw);
    f->head = 0;
    f->seen = 0;
}

/* Fir::apply (fir.rs:23-32): pop_back, push_front(value), then
 *   accum = 0; for (c, v) in coef.zip(buffer) { accum += v * c }
 * buffer[0] is the newest sample.  The doubled ring keeps buffer[k] = ring[head+k]
 * contiguous; arithmetic order is unchanged. */
static inline void fir_push(oracle_fir* f, const float* x) {
    size_t K = f->K;
    f->head = (f->head == 0) ? K - 1 : f->head - 1;
    if (f->sk == ORACLE_C64) {
        f->ring[2 * f->head] = x[0]; f->ring[2 * f->head + 1] = x[1];
        f->ring[2 * (f->head + K)] = x[0]; f->ring[2 * (f->head + K) + 1] = x[1];
    } else {
        f->ring[f->head] = x[0]; f->ring[f->head + K] = x[0];
    }
}

static inline void fir_dot(const oracle_fir* f, float* y) {
    size_t K = f->K;
    if (f->sk == ORACLE_F32) {
        const float* b = f->ring + f->head;
        float acc = 0.0f;
        for (size_t k = 0; k < K; ++k) acc += b[k] * f->taps[k];
        y[0] = acc;
    } else if (f->tk == ORACLE_F32) {
        const c32* b = (const c32*)(f->ring) + f->head;
        c32 acc = {0.0f, 0.0f};
        for (size_t k = 0; k < K; ++k) {
            c32 p = cmul_r(b[k], f->taps[k]);
            acc.re += p.re; acc.im += p.im;
        }
        y[0] = acc.re; y[1] = acc.im;
    } else {
        const c32* b = (const c32*)(f->ring) + f->head;
        const c32* h = (const c32*)f->taps;
        c32 acc = {0.0f, 0.0f};
        for (size_t k = 0; k < K; ++k) {
            c32 p = cmul(b[k], h[k]);
            acc.re += p.re; acc.im += p.im;
        }
        y[0] = acc.re; y[1] = acc.im;
    }
}

/* Signal::filter(taps).decimate(rate) (signal/mod.rs:26-28,42-48; adapters/mod.rs:30-37):
 * every input runs Fir::apply; Decimate keeps upstream indices wait-1, 2wait-1, ... */
size_t oracle_fir_process(oracle_fir* f, const float* in, size_t n_in, float* out) {
    size_t sw = (f->sk == ORACLE_C64) ? 2 : 1;
    size_t n_out = 0;
    float y[2];
    for (size_t i = 0; i < n_in; ++i) {
        fir_push(f, in + i * sw);
        fir_dot(f, y);           /* the reference computes every output */
        f->seen++;
        if (f->seen % f->D == 0) {
            memcpy(out + n_out * sw, y, sizeof(float) * sw);
            n_out++;
        }
    }
    return n_out;
}

typedef struct {
    int sk, tk; const float* taps; size_t ntaps; uint32_t D;
    const float* in; size_t ld_in; size_t n_in; float* out; size_t ld_out;
    size_t ch0, ch1; size_t n_out;
} fir_job;

static void* fir_job_run(void* arg) {
    fir_job* j = (fir_job*)arg;
    size_t sw = (j->sk == ORACLE_C64) ? 2 : 1;
    oracle_fir* f = oracle_fir_create(j->sk, j->tk, j->taps, j->ntaps, j->D);
    for (size_t c = j->ch0; c < j->ch1; ++c) {
        oracle_fir_reset(f);
        j->n_out = oracle_fir_process(f, j->in + c * j->ld_in * sw, j->n_in,
                                      j->out + c * j->ld_out * sw);
    }
    oracle_fir_destroy(f);
    return NULL;
}

size_t oracle_fir_batch(int sk, int tk, const float* taps, size_t ntaps, uint32_t D,
                        size_t nch, const float* in, size_t ld_in, size_t n_in,
                        float* out, size_t ld_out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > nch) nthreads = (int)(nch ? nch : 1);
    pthread_t th[256];
    fir_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; ++t) {
        fir_job* j = &jobs[t];
        j->sk = sk; j->tk = tk; j->taps = taps; j->ntaps = ntaps; j->D = D;
        j->in = in; j->ld_in = ld_in; j->n_in = n_in; j->out = out; j->ld_out = ld_out;
        j->ch0 = nch * t / nthreads; j->ch1 = nch * (t + 1) / nthreads; j->n_out = 0;
        pthread_create(&th[t], NULL, fir_job_run, j);
    }
    size_t n_out = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].ch1 > jobs[t].ch0) n_out = jobs[t].n_out;
    }
    return n_out;
}

/* ================================ Biquad ================================ */
/* BiquadD::design (biquad.rs:83-155) then Biquad::new (:25-38).  All f32. */
static const float PI_F = 3.14159265358979323846f; /* std::f32::consts::PI */

static void bq_new(float a0, float a1, float a2, float b0, float b1, float b2,
                   oracle_biquad_coefs* c) {
    c->b0 = b0 / a0;
    c->b1 = b1 / a0;
    c->b2 = b2 / a0;
    c->na1 = -a1 / a0;
    c->na2 = -a2 / a0;
}

void oracle_biquad_design_coefs(oracle_biquad_design d, float rate, oracle_biquad_coefs* c) {
    float omega, cs, alpha;
    switch (d.kind) {
    case ORACLE_BQ_LOWPASS:   /* biquad.rs:89-101 */
        omega = 2.0f * PI_F * d.freq / rate;
        cs = cosf(omega);
        alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, (1.0f - cs) / 2.0f, 1.0f - cs,
               (1.0f - cs) / 2.0f, c);
        break;
    case ORACLE_BQ_HIGHPASS:  /* biquad.rs:102-114 */
        omega = 2.0f * PI_F * d.freq / rate;
        cs = cosf(omega);
        alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, (1.0f + cs) / 2.0f, -1.0f - cs,
               (1.0f + cs) / 2.0f, c);
        break;
    case ORACLE_BQ_BANDPASS:  /* biquad.rs:115-127 */
        omega = 2.0f * PI_F * d.freq / rate;
        cs = cosf(omega);
        alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, alpha, 0.0f, -alpha, c);
        break;
    case ORACLE_BQ_NOTCH:     /* biquad.rs:128-140 */
        omega = 2.0f * PI_F * d.freq / rate;
        cs = cosf(omega);
        alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, 1.0f, -2.0f * cs, 1.0f, c);
        break;
    case ORACLE_BQ_LR: {      /* biquad.rs:141-151 */
        float decayn = d.freq / rate;
        bq_new(1.0f, -expf(-decayn), 0.0f, decayn, 0.0f, 0.0f, c);
        break;
    }
    default:                  /* Identity: y = x, represented as b0 = 1 */
        c->b0 = 1.0f; c->b1 = 0.0f; c->b2 = 0.0f; c->na1 = 0.0f; c->na2 = 0.0f;
        break;
    }
}

typedef struct { oracle_biquad_coefs c; float x1, x2, y1, y2; int ident; } bq_r;
typedef struct { oracle_biquad_coefs c; c32 x1, x2, y1, y2; } bq_c;

/* Biquad::apply (biquad.rs:43-56): out = 0; out += v*b0; += x1*b1; += x2*b2;
 * += y1*na1; += y2*na2; then x2 <- x1, x1 <- v, y2 <- y1, y1 <- out. */
static inline float bq_r_apply(bq_r* s, float v) {
    if (s->ident) return v;
    float out = 0.0f;
    out += v * s->c.b0;
    out += s->x1 * s->c.b1;
    out += s->x2 * s->c.b2;
    out += s->y1 * s->c.na1;
    out += s->y2 * s->c.na2;
    s->x2 = s->x1; s->x1 = v;
    s->y2 = s->y1; s->y1 = out;
    return out;
}

static inline c32 bq_c_apply(bq_c* s, c32 v) {
    c32 out = {0.0f, 0.0f}, p;
    p = cmul_r(v, s->c.b0);     out.re += p.re; out.im += p.im;
    p = cmul_r(s->x1, s->c.b1); out.re += p.re; out.im += p.im;
    p = cmul_r(s->x2, s->c.b2); out.re += p.re; out.im += p.im;
    p = cmul_r(s->y1, s->c.na1); out.re += p.re; out.im += p.im;
    p = cmul_r(s->y2, s->c.na2); out.re += p.re; out.im += p.im;
    s->x2 = s->x1; s->x1 = v;
    s->y2 = s->y1; s->y1 = out;
    return out;
}

void oracle_biquad_run(oracle_biquad_design d, float rate, int sk, const float* in,
                       size_t n, float* out) {
    if (sk == ORACLE_F32) {
        bq_r s; memset(&s, 0, sizeof(s));
        oracle_biquad_design_coefs(d, rate, &s.c);
        s.ident = (d.kind == ORACLE_BQ_IDENTITY);
        for (size_t i = 0; i < n; ++i) out[i] = bq_r_apply(&s, in[i]);
    } else {
        bq_c s; memset(&s, 0, sizeof(s));
        oracle_biquad_design_coefs(d, rate, &s.c);
        const c32* x = (const c32*)in; c32* y = (c32*)out;
        if (d.kind == ORACLE_BQ_IDENTITY) { memcpy(out, in, n * sizeof(c32)); return; }
        for (size_t i = 0; i < n; ++i) y[i] = bq_c_apply(&s, x[i]);
    }
}

/* ================================ PLL ================================== */
typedef struct {
    float rate, reference, gain;
    bq_c loopf; bq_r outf, lockf;
    float nphase; c32 value;
} pll_state;

/* PllDesign::design (pll.rs:48-60) */
static void pll_design(const oracle_pll_params* p, pll_state* s) {
    memset(s, 0, sizeof(*s));
    s->rate = p->rate;
    s->reference = p->reference / p->rate;
    s->gain = p->gain;
    oracle_biquad_design_coefs(p->loopf, p->rate, &s->loopf.c);
    oracle_biquad_design_coefs(p->outputf, p->rate, &s->outf.c);
    s->outf.ident = (p->outputf.kind == ORACLE_BQ_IDENTITY);
    oracle_biquad_design_coefs(p->lockf, p->rate, &s->lockf.c);
    s->lockf.ident = (p->lockf.kind == ORACLE_BQ_IDENTITY);
    s->nphase = 0.0f;
    s->value.re = 0.0f; s->value.im = 0.0f;
}

/* Pll::apply (pll.rs:70-85). */
static inline float pll_apply(pll_state* s, c32 x, uint8_t* locked_out, int loop_ident) {
    c32 conjv = {s->value.re, -s->value.im};
    c32 c = cmul(x, conjv);                                    /* :71 */
    c32 lf = loop_ident ? c : bq_c_apply(&s->loopf, c);
    float phasedif = atan2f(lf.im, lf.re) * s->gain;           /* :72 arg() */
    s->nphase += s->reference + phasedif;                      /* :73 */
    s->nphase = s->nphase - truncf(s->nphase);                 /* :74 fract() */
    float phase = 2.0f * PI_F * s->nphase;                     /* :75 */
    s->value.re = 1.0f * cosf(phase);                          /* :76 from_polar */
    s->value.im = 1.0f * sinf(phase);
    float locked = bq_r_apply(&s->lockf, c.re);                /* :78 */
    float output = bq_r_apply(&s->outf, phasedif * s->rate);   /* :79 */
    if (locked > 0.01f) { *locked_out = 1; return output; }    /* :80-84 */
    *locked_out = 0;
    return 0.0f;                                               /* main.rs:49 */
}

/* src/main.rs:56-69: the stereo pilot map over a real stream v (one channel):
 * mono = v * 0.5; diff = Some -> (v / value.powi(2)).re * 0.5, None -> 0.0, where
 * pllpilot.apply(Complex::new(v, 0.0)) updated `value`.  num-complex 0.2: powi(2) =
 * value * value; f32 / Complex -> re = v * w.re / w.norm_sqr(). */
void oracle_pll_stereo(const oracle_pll_params* p, const float* v, size_t n, float* mono,
                       float* diff, uint8_t* locked) {
    pll_state s; pll_design(p, &s);
    const int loop_ident = p->loopf.kind == ORACLE_BQ_IDENTITY;
    for (size_t i = 0; i < n; ++i) {
        c32 x = {v[i], 0.0f};
        (void)pll_apply(&s, x, &locked[i], loop_ident);
        mono[i] = v[i] * 0.5f;
        if (locked[i]) {
            c32 w = cmul(s.value, s.value);
            float nrm = w.re * w.re + w.im * w.im;
            diff[i] = v[i] * w.re / nrm * 0.5f;
        } else {
            diff[i] = 0.0f;
        }
    }
}

typedef struct {
    const oracle_pll_params* p; const float* in; size_t ld_in, n; float* out;
    uint8_t* locked; size_t ld_out; size_t ch0, ch1;
} pll_job;

static void* pll_job_run(void* arg) {
    pll_job* j = (pll_job*)arg;
    int loop_ident = (j->p->loopf.kind == ORACLE_BQ_IDENTITY);
    for (size_t c = j->ch0; c < j->ch1; ++c) {
        pll_state s; pll_design(j->p, &s);
        const c32* x = (const c32*)j->in + c * j->ld_in;
        float* y = j->out + c * j->ld_out;
        uint8_t* lk = j->locked + c * j->ld_out;
        for (size_t i = 0; i < j->n; ++i) y[i] = pll_apply(&s, x[i], &lk[i], loop_ident);
    }
    return NULL;
}

void oracle_pll_batch(const oracle_pll_params* p, size_t nch, const float* in,
                      size_t ld_in, size_t n, float* out, uint8_t* locked,
                      size_t ld_out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > nch) nthreads = (int)(nch ? nch : 1);
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256]; pll_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        pll_job* j = &jobs[t];
        j->p = p; j->in = in; j->ld_in = ld_in; j->n = n; j->out = out;
        j->locked = locked; j->ld_out = ld_out;
        j->ch0 = nch * t / nthreads; j->ch1 = nch * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, pll_job_run, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* ================================ FFT ================================== */
typedef struct { double re, im; } c64d;

static void dft_f64(c64d* a, size_t n) {
    if (n == 0) return;
    if ((n & (n - 1)) == 0) {
        /* iterative radix-2 DIT, forward (sign -1) like rustfft FFTplanner::new(false) */
        for (size_t i = 1, j = 0; i < n; ++i) {
            size_t bit = n >> 1;
            for (; j & bit; bit >>= 1) j ^= bit;
            j ^= bit;
            if (i < j) { c64d t = a[i]; a[i] = a[j]; a[j] = t; }
        }
        for (size_t len = 2; len <= n; len <<= 1) {
            double ang = -2.0 * M_PI / (double)len;
            for (size_t i = 0; i < n; i += len) {
                for (size_t k = 0; k < len / 2; ++k) {
                    double wr = cos(ang * (double)k), wi = sin(ang * (double)k);
                    c64d u = a[i + k], v = a[i + k + len / 2];
                    c64d t = {v.re * wr - v.im * wi, v.re * wi + v.im * wr};
                    a[i + k].re = u.re + t.re; a[i + k].im = u.im + t.im;
                    a[i + k + len / 2].re = u.re - t.re; a[i + k + len / 2].im = u.im - t.im;
                }
            }
        }
    } else {
        /* direct DFT (any n): W_n^m from a table of the same f64 cos/sin values */
        c64d* t = (c64d*)malloc(sizeof(c64d) * n);
        double* cs = (double*)malloc(sizeof(double) * 2 * n);
        for (size_t m = 0; m < n; ++m) {
            double ang = -2.0 * M_PI * (double)m / (double)n;
            cs[2 * m] = cos(ang);
            cs[2 * m + 1] = sin(ang);
        }
        for (size_t k = 0; k < n; ++k) {
            double sr = 0, si = 0;
            size_t m = 0;
            for (size_t j = 0; j < n; ++j) {
                double c = cs[2 * m], sn = cs[2 * m + 1];
                sr += a[j].re * c - a[j].im * sn;
                si += a[j].re * sn + a[j].im * c;
                m += k;
                if (m >= n) m -= n;
            }
            t[k].re = sr; t[k].im = si;
        }
        memcpy(a, t, sizeof(c64d) * n);
        free(cs);
        free(t);
    }
}

/* fft::fft collate (fft.rs:14-26): out[i] = X[(i - n/2) mod n] * (1/sqrt(n)) in f32. */
void oracle_fft_frame(const float* in, size_t n, float* out) {
    c64d* a = (c64d*)malloc(sizeof(c64d) * (n ? n : 1));
    for (size_t i = 0; i < n; ++i) { a[i].re = in[2 * i]; a[i].im = in[2 * i + 1]; }
    dft_f64(a, n);
    float norm = 1.0f / sqrtf((float)n);
    long start = -(long)(n / 2);
    for (size_t i = 0; i < n; ++i) {
        long srci = start + (long)i;
        size_t pos = (size_t)(srci < 0 ? srci + (long)n : srci);
        float re = (float)a[pos].re, im = (float)a[pos].im;
        out[2 * i] = re * norm;
        out[2 * i + 1] = im * norm;
    }
    free(a);
}

typedef struct {
    const float* in; size_t n_in, n, hop; float* out; size_t f0, f1;
} stft_job;

static void* stft_job_run(void* arg) {
    stft_job* j = (stft_job*)arg;
    float* frame = (float*)malloc(sizeof(float) * 2 * j->n);
    for (size_t f = j->f0; f < j->f1; ++f) {
        long end = (long)((f + 1) * j->hop);          /* exclusive */
        long beg = end - (long)j->n;
        for (size_t i = 0; i < j->n; ++i) {
            long g = beg + (long)i;
            if (g < 0) { frame[2 * i] = 0.0f; frame[2 * i + 1] = 0.0f; }
            else { frame[2 * i] = j->in[2 * g]; frame[2 * i + 1] = j->in[2 * g + 1]; }
        }
        oracle_fft_frame(frame, j->n, j->out + f * 2 * j->n);
    }
    free(frame);
    return NULL;
}

/* Window::next keeps the last cap samples, zero-prefilled (adapters/mod.rs:277-299);
 * Decimate(wait=hop) yields it after inputs hop-1, 2hop-1, ... (:30-37). */
size_t oracle_stft(const float* in, size_t n_in, size_t n, size_t hop, float* out,
                   size_t max_frames, int nthreads) {
    size_t nf = n_in / hop;
    if (nf > max_frames) nf = max_frames;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > nf) nthreads = (int)(nf ? nf : 1);
    pthread_t th[256]; stft_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        stft_job* j = &jobs[t];
        j->in = in; j->n_in = n_in; j->n = n; j->hop = hop; j->out = out;
        j->f0 = nf * t / nthreads; j->f1 = nf * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, stft_job_run, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return nf;
}

/* ================================ Sources =============================== */
/* Freq -> FreqSweep::new(rate, f, 0, phase, 0, 0, None) (sources.rs:129-143,203-207)
 * and FreqSweep::next (:150-175) with dfdt forced to 0. */
void oracle_freq(float rate, float freq, float phase, size_t n, float* out) {
    float dt = 1.0f / rate;
    float f = freq;
    float nphase = phase / (2.0f * PI_F);
    for (size_t i = 0; i < n; ++i) {
        float dfdt = 0.0f;
        f += dt * dfdt;
        nphase += dt * f;
        nphase = nphase - truncf(nphase);
        float ph = 2.0f * PI_F * nphase;
        out[2 * i] = 1.0f * cosf(ph);
        out[2 * i + 1] = 1.0f * sinf(ph);
    }
}

/* `value.round() as usize` (Rust): round half away from zero, saturating at 0 (and NaN -> 0) */
static size_t f32_round_usize(float v) {
    float r = roundf(v);
    if (!(r > 0.0f)) return 0;
    if (r >= 18446744073709551616.0f) return (size_t)-1;
    return (size_t)r;
}

/* freq_sweep(rate, df, warmup, start..end) (sources.rs:181-194): dfdt = df.powi(2) (negated
 * for a falling sweep), endt = (end - start) / dfdt, warmupt = warmup ? 1/df : 0, then
 * FreqSweep::new(rate, start, dfdt, 0.0, warmupt, warmupt + endt, Some(warmupt + endt))
 * (:129-143) and FreqSweep::next (:146-174).  Writes at most `cap` samples (freq, value) and
 * returns the sweep's length. */
size_t oracle_freq_sweep(float rate, float df, int warmup, float start, float end, size_t cap,
                         float* freqs, float* out) {
    float dfdt = df * df;
    if (start > end) dfdt = -dfdt;
    float endt = (end - start) / dfdt;
    float warmupt = warmup ? 1.0f / df : 0.0f;
    float fend_t = warmupt + endt;
    float dt = 1.0f / rate;
    float f = start;
    float nphase = 0.0f / (2.0f * PI_F);
    size_t fstart = f32_round_usize(warmupt * rate);
    size_t fend = f32_round_usize(fend_t * rate);
    size_t length = f32_round_usize(fend_t * rate);
    size_t total = length;
    for (size_t i = 0; i < total && i < cap; ++i) {
        float d = dfdt;
        if (fstart > 0) {
            fstart -= 1;
            d = 0.0f;
        }
        if (fend > 0) fend -= 1;
        else d = 0.0f;
        f += dt * d;
        nphase += dt * f;
        nphase = nphase - truncf(nphase);
        float ph = 2.0f * PI_F * nphase;
        freqs[i] = f;
        out[2 * i] = 1.0f * cosf(ph);
        out[2 * i + 1] = 1.0f * sinf(ph);
    }
    return total;
}

/* Host glibc atan2f (fn 0) or sinf / cosf (fn 1) over n arguments: what Rust's f32::atan2 /
 * sin / cos call on x86-64 Linux (pll.rs:71-78); the checker for the device restatements in
 * libm_glibc.h (tests/test_libm_gpu.py). */
void oracle_libm(int fn, const float* a, const float* b, float* out0, float* out1, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        if (fn == 0) {
            out0[i] = atan2f(a[i], b[i]);
        } else {
            out0[i] = sinf(a[i]);
            out1[i] = cosf(a[i]);
        }
    }
}

/* RtlTcpSignal::next (rtltcp.rs:156-164): (v - 128) / 128 */
void oracle_u8_to_c64(const uint8_t* in, size_t n, float* out) {
    for (size_t i = 0; i < 2 * n; ++i) out[i] = ((float)in[i] - 128.0f) / 128.0f;
}

/* ======================= sample-rate conversion (libsamplerate) =====================
 * src/resample.rs:46-67 fills an SRC_DATA and calls src_process; restated here are
 * samplerate.c's src_process checks and src_zoh.c / src_linear.c's process loops, counting
 * in samples (frames x channels) as those files do. */
typedef struct sinc_filter sinc_filter;
struct oracle_src {
    int converter, channels, reset;
    double last_ratio, last_position;
    float* last_value;
    sinc_filter* sinc; /* converters 0..2 */
};
static sinc_filter* sinc_new(int converter, int channels);
static void sinc_free(sinc_filter* f);
static void sinc_reset(sinc_filter* f);
static int sinc_process(oracle_src* s, const float* in, long in_frames, float* out,
                        long out_frames, double ratio, long* in_used_frames, long* out_gen_frames);

static double src_fmod_one(double x) {
    double res = x - lrint(x);
    if (res < 0.0) return res + 1.0;
    return res;
}

static int src_bad_ratio(double r) { return r < (1.0 / 256.0) || r > 256.0; }

oracle_src* oracle_src_new(int converter, int channels, int* error) {
    *error = 0;
    if (converter < 0 || converter > 4) { *error = 10; return NULL; }
    if (channels < 1) { *error = 11; return NULL; }
    oracle_src* s = (oracle_src*)calloc(1, sizeof(*s));
    s->converter = converter;
    s->channels = channels;
    s->last_value = (float*)calloc((size_t)channels, sizeof(float));
    if (converter <= 2) s->sinc = sinc_new(converter, channels);
    oracle_src_reset(s);
    return s;
}

void oracle_src_delete(oracle_src* s) {
    if (!s) return;
    sinc_free(s->sinc);
    free(s->last_value);
    free(s);
}

int oracle_src_reset(oracle_src* s) {
    s->reset = 1;
    memset(s->last_value, 0, sizeof(float) * (size_t)s->channels);
    s->last_position = 0.0;
    s->last_ratio = 0.0;
    if (s->sinc) sinc_reset(s->sinc);
    return 0;
}

int oracle_src_set_ratio(oracle_src* s, double ratio) {
    if (src_bad_ratio(ratio)) return 6;
    s->last_ratio = ratio;
    return 0;
}

int oracle_src_process(oracle_src* s, const float* in, long in_frames, float* out,
                       long out_frames, double ratio, long* in_used_frames, long* out_gen_frames) {
    *in_used_frames = 0;
    *out_gen_frames = 0;
    if ((in == NULL && in_frames > 0) || (out == NULL && out_frames > 0)) return 4;
    if (src_bad_ratio(ratio)) return 6;
    if (in_frames < 0) in_frames = 0;
    if (out_frames < 0) out_frames = 0;
    if (s->last_ratio < (1.0 / 256.0)) s->last_ratio = ratio;
    if (s->sinc) return sinc_process(s, in, in_frames, out, out_frames, ratio, in_used_frames,
                                     out_gen_frames);
    /* converter process loop */
    if (in_frames <= 0) return 0;
    const int ch = s->channels, linear = s->converter == 4;
    if (s->reset) {
        for (int c = 0; c < ch; c++) s->last_value[c] = in[c];
        s->reset = 0;
    }
    long in_count = in_frames * ch, out_count = out_frames * ch, in_used = 0, out_gen = 0;
    double src_ratio = s->last_ratio, input_index, rem;
    if (src_bad_ratio(src_ratio)) return 22;
    input_index = s->last_position;
    while (input_index < 1.0 && out_gen < out_count) {
        if (linear) {
            if (in_used + ch * (1.0 + input_index) >= in_count) break;
        } else {
            if (in_used + ch * input_index >= in_count) break;
        }
        if (out_count > 0 && fabs(s->last_ratio - ratio) > 1e-20)
            src_ratio = s->last_ratio + out_gen * (ratio - s->last_ratio) / out_count;
        for (int c = 0; c < ch; c++) {
            if (linear)
                out[out_gen] = (float)(s->last_value[c] +
                                       input_index * ((double)in[c] - s->last_value[c]));
            else
                out[out_gen] = s->last_value[c];
            out_gen++;
        }
        input_index += 1.0 / src_ratio;
    }
    rem = src_fmod_one(input_index);
    in_used += ch * lrint(input_index - rem);
    input_index = rem;
    while (out_gen < out_count &&
           (linear ? in_used + ch * input_index < in_count
                   : in_used + ch * input_index <= in_count)) {
        if (out_count > 0 && fabs(s->last_ratio - ratio) > 1e-20)
            src_ratio = s->last_ratio + out_gen * (ratio - s->last_ratio) / out_count;
        for (int c = 0; c < ch; c++) {
            /* in_used == 0 here (a 1-frame block with input_index in (0, 1), the case
             * libsamplerate's SRC_DEBUG "Whoops" check flags): the frame before data_in[0]
             * is last_value, where libsamplerate would read data_in[-channels]. */
            const float left = in_used >= ch ? in[in_used - ch + c] : s->last_value[c];
            if (linear)
                out[out_gen] = (float)(left + input_index * ((double)in[in_used + c] - left));
            else
                out[out_gen] = left;
            out_gen++;
        }
        input_index += 1.0 / src_ratio;
        rem = src_fmod_one(input_index);
        in_used += ch * lrint(input_index - rem);
        input_index = rem;
    }
    if (in_used > in_count) {
        input_index += (in_used - in_count) / ch;
        in_used = in_count;
    }
    s->last_position = input_index;
    if (in_used > 0)
        for (int c = 0; c < ch; c++) s->last_value[c] = in[in_used - ch + c];
    s->last_ratio = src_ratio;
    *in_used_frames = in_used / ch;
    *out_gen_frames = out_gen / ch;
    return 0;
}

/* ======================= sinc converters (libsamplerate src_sinc.c) ===================
 * SincBestQuality / SincMediumQuality / SincFastest (ids 0 / 1 / 2, src/resample.rs:
 * 112-149; src/main.rs:50 uses SincFastest, Signal::resample SincBestQuality,
 * src/signal/mod.rs:78-84).  Restated from libsamplerate 0.2's published src_sinc.c:
 * sinc_set_converter (buffer length), sinc_reset, prepare_data (the input ring with its
 * zero lead-in, memmove compaction and end-of-input zero tail), the vari process loop
 * (fixed-point filter index, 12 fraction bits; ratio ramp; termination) and
 * calc_output_multi (left half walked outward-in, right half inward-out, each tap's
 * coefficient linearly interpolated between table entries, f64 accumulation).
 *
 * The coefficient TABLES of libsamplerate (fastest_coeffs.h, mid_qual_coeffs.h,
 * high_qual_coeffs.h) are not in this image; the tables here keep their increments and
 * lengths (128 / 2464, 491 / 22438, 2381 / 340239) and are our own Kaiser-windowed sincs
 * (oracle_sinc_table).  So outputs follow libsamplerate's algorithm with a different
 * low-pass: parity is UNPINNED for the sinc converters. */

#define SINC_SHIFT_BITS 12
#define SINC_FP_ONE ((double)(1 << SINC_SHIFT_BITS))
#define SINC_INV_FP_ONE (1.0 / SINC_FP_ONE)

static const struct { int inc, len; double atten_db; } k_sinc_spec[3] = {
    {2381, 340239, 144.0}, /* best    */
    {491, 22438, 121.0},   /* medium  */
    {128, 2464, 97.0},     /* fastest */
};

static double bessel_i0(double x) {
    double sum = 1.0, term = 1.0, q = 0.25 * x * x;
    for (int k = 1; k < 500; k++) {
        term *= q / ((double)k * (double)k);
        sum += term;
        if (term < 1e-17 * sum) break;
    }
    return sum;
}

/* Kaiser-windowed sinc sampled at t = i / inc input samples (i < len; zero at and beyond
 * the half length T = (len - 2) / inc).  Kaiser's formulas for attenuation A over the
 * window length 2T: transition width dw = (A - 8) / (2.285 * 2T) rad/sample, stopband edge
 * at Nyquist, cutoff fc = 1 - dw / (2 pi) (Nyquist units), beta = 0.1102 (A - 8.7); the
 * table is scaled so the integer-spaced taps sum to 1 (unit DC gain at ratio >= 1). */
int oracle_sinc_table(int converter, float* out, int cap, int* increment) {
    if (converter < 0 || converter > 2) return -1;
    const int inc = k_sinc_spec[converter].inc, len = k_sinc_spec[converter].len;
    if (increment) *increment = inc;
    if (!out) return len;
    if (cap < len) return -1;
    const double A = k_sinc_spec[converter].atten_db;
    const double T = (double)(len - 2) / (double)inc;
    const double dw = (A - 8.0) / (2.285 * 2.0 * T);
    const double fc = 1.0 - dw / (2.0 * M_PI);
    const double beta = 0.1102 * (A - 8.7), i0b = bessel_i0(beta);
    double* h = (double*)malloc(sizeof(double) * (size_t)len);
    if (!h) return -1;
    for (int i = 0; i < len; i++) {
        const double t = (double)i / (double)inc;
        if (t >= T) { h[i] = 0.0; continue; }
        const double x = t / T;
        const double w = bessel_i0(beta * sqrt(1.0 - x * x)) / i0b;
        const double s = i == 0 ? fc : sin(M_PI * fc * t) / (M_PI * t);
        h[i] = s * w;
    }
    double g = len > 0 ? h[0] : 1.0;
    for (int i = inc; i < len; i += inc) g += 2.0 * h[i];
    for (int i = 0; i < len; i++) out[i] = (float)(h[i] / g);
    free(h);
    return len;
}

struct sinc_filter {
    int channels;
    long in_count, in_used, out_count, out_gen;
    int coeff_half_len, index_inc;
    float* coeffs;
    int b_current, b_end, b_real_end, b_len;
    float* buffer; /* b_len + channels */
    double *left, *right;
};

static sinc_filter* sinc_new(int converter, int channels) {
    sinc_filter* f = (sinc_filter*)calloc(1, sizeof(*f));
    int inc = 0;
    const int len = oracle_sinc_table(converter, NULL, 0, &inc);
    f->channels = channels;
    f->coeffs = (float*)malloc(sizeof(float) * (size_t)len);
    oracle_sinc_table(converter, f->coeffs, len, &inc);
    f->coeff_half_len = len - 2; /* ARRAY_LEN (coeffs) - 2 */
    f->index_inc = inc;
    /* sinc_set_converter */
    int b_len = 3 * (int)lrint((f->coeff_half_len + 2.0) / f->index_inc * 256.0 + 1);
    if (b_len < 4096) b_len = 4096;
    b_len *= channels;
    b_len += 1;
    f->b_len = b_len;
    f->buffer = (float*)calloc((size_t)(b_len + channels), sizeof(float));
    f->left = (double*)calloc((size_t)channels, sizeof(double));
    f->right = (double*)calloc((size_t)channels, sizeof(double));
    sinc_reset(f);
    return f;
}

static void sinc_free(sinc_filter* f) {
    if (!f) return;
    free(f->coeffs);
    free(f->buffer);
    free(f->left);
    free(f->right);
    free(f);
}

static void sinc_reset(sinc_filter* f) {
    f->b_current = f->b_end = 0;
    f->b_real_end = -1;
    memset(f->buffer, 0, sizeof(float) * (size_t)f->b_len);
}

/* prepare_data: fill the buffer from data_in (never NULL from Rust; end_of_input is
 * input.len() == 0, src/resample.rs:53). */
static int sinc_prepare_data(sinc_filter* f, const float* in, int end_of_input, int half) {
    const int ch = f->channels;
    int len = 0;
    if (f->b_real_end >= 0) return 0; /* terminating */
    if (f->b_current == 0) {
        len = f->b_len - 2 * half; /* initial: zeros lead in, load after them */
        f->b_current = f->b_end = half;
    } else if (f->b_end + half + ch < f->b_len) {
        len = f->b_len - f->b_current - half;
        if (len < 0) len = 0;
    } else {
        len = f->b_end - f->b_current;
        if (f->b_current - half < 0) return 21; /* would read before the buffer */
        memmove(f->buffer, f->buffer + f->b_current - half, sizeof(float) * (size_t)(half + len));
        f->b_current = half;
        f->b_end = f->b_current + len;
        len = f->b_len - f->b_current - half;
        if (len < 0) len = 0;
    }
    if ((long)len > f->in_count - f->in_used) len = (int)(f->in_count - f->in_used);
    len -= len % ch;
    if (len < 0 || f->b_end + len > f->b_len) return 21; /* SINC_PREPARE_DATA_BAD_LEN */
    if (len) memcpy(f->buffer + f->b_end, in + f->in_used, sizeof(float) * (size_t)len);
    f->b_end += len;
    f->in_used += len;
    if (f->in_used == f->in_count && f->b_end - f->b_current < 2 * half && end_of_input) {
        if (f->b_len - f->b_end < half + 5) {
            len = f->b_end - f->b_current;
            if (f->b_current - half < 0) return 21;
            memmove(f->buffer, f->buffer + f->b_current - half, sizeof(float) * (size_t)(half + len));
            f->b_current = half;
            f->b_end = f->b_current + len;
        }
        f->b_real_end = f->b_end;
        len = half + 5;
        if (len < 0 || f->b_end + len > f->b_len) len = f->b_len - f->b_end;
        memset(f->buffer + f->b_end, 0, sizeof(float) * (size_t)len);
        f->b_end += len;
    }
    return 0;
}

/* calc_output_multi: one output frame at b_current + input_index */
static void sinc_calc_output(sinc_filter* f, int increment, int start_filter_index,
                             double scale, float* out) {
    const int ch = f->channels;
    const int max_filter_index = f->coeff_half_len << SINC_SHIFT_BITS;
    const float* c = f->coeffs;
    /* left half */
    int filter_index = start_filter_index;
    int coeff_count = (max_filter_index - filter_index) / increment;
    filter_index = filter_index + coeff_count * increment;
    int data_index = f->b_current - ch * coeff_count;
    if (data_index < 0) { /* avoid reading before the buffer */
        const int steps = (-data_index + ch - 1) / ch;
        filter_index -= increment * steps;
        data_index += steps * ch;
    }
    for (int k = 0; k < ch; k++) f->left[k] = 0.0;
    while (filter_index >= 0) {
        const double fraction = (double)(filter_index & ((1 << SINC_SHIFT_BITS) - 1)) * SINC_INV_FP_ONE;
        const int indx = filter_index >> SINC_SHIFT_BITS;
        const double icoeff = c[indx] + fraction * (c[indx + 1] - c[indx]);
        for (int k = 0; k < ch; k++) f->left[k] += icoeff * f->buffer[data_index + k];
        filter_index -= increment;
        data_index = data_index + ch;
    }
    /* right half */
    filter_index = increment - start_filter_index;
    coeff_count = (max_filter_index - filter_index) / increment;
    filter_index = filter_index + coeff_count * increment;
    data_index = f->b_current + ch * (1 + coeff_count);
    for (int k = 0; k < ch; k++) f->right[k] = 0.0;
    do {
        const double fraction = (double)(filter_index & ((1 << SINC_SHIFT_BITS) - 1)) * SINC_INV_FP_ONE;
        const int indx = filter_index >> SINC_SHIFT_BITS;
        const double icoeff = c[indx] + fraction * (c[indx + 1] - c[indx]);
        for (int k = 0; k < ch; k++) f->right[k] += icoeff * f->buffer[data_index + k];
        filter_index -= increment;
        data_index = data_index - ch;
    } while (filter_index > 0);
    for (int k = 0; k < ch; k++) out[k] = (float)(scale * (f->left[k] + f->right[k]));
}

/* sinc_multichan_vari_process (const and vari process are the same loop) */
static int sinc_process(oracle_src* s, const float* in, long in_frames, float* out,
                        long out_frames, double ratio, long* in_used_frames, long* out_gen_frames) {
    sinc_filter* f = s->sinc;
    const int ch = f->channels;
    f->in_count = in_frames * ch;
    f->out_count = out_frames * ch;
    f->in_used = f->out_gen = 0;
    double src_ratio = s->last_ratio;
    if (src_bad_ratio(src_ratio)) return 22;
    double count = (f->coeff_half_len + 2.0) / f->index_inc;
    const double rmin = s->last_ratio < ratio ? s->last_ratio : ratio;
    if (rmin < 1.0) count /= rmin;
    const int half = ch * ((int)lrint(count) + 1);
    double input_index = s->last_position;
    double rem = src_fmod_one(input_index);
    f->b_current = (f->b_current + ch * (int)lrint(input_index - rem)) % f->b_len;
    input_index = rem;
    const double terminate = 1.0 / src_ratio + 1e-20;
    const int end_of_input = in_frames == 0;
    while (f->out_gen < f->out_count) {
        int in_hand = (f->b_end - f->b_current + f->b_len) % f->b_len;
        if (in_hand <= half) {
            const int err = sinc_prepare_data(f, in, end_of_input, half);
            if (err) return err;
            in_hand = (f->b_end - f->b_current + f->b_len) % f->b_len;
            if (in_hand <= half) break;
        }
        if (f->b_real_end >= 0 && f->b_current + input_index + terminate > f->b_real_end) break;
        if (f->out_count > 0 && fabs(s->last_ratio - ratio) > 1e-10)
            src_ratio = s->last_ratio + f->out_gen * (ratio - s->last_ratio) / f->out_count;
        const double float_increment = f->index_inc * (src_ratio < 1.0 ? src_ratio : 1.0);
        const int increment = (int)lrint(float_increment * SINC_FP_ONE);
        const int start_filter_index = (int)lrint(input_index * float_increment * SINC_FP_ONE);
        sinc_calc_output(f, increment, start_filter_index, float_increment / f->index_inc,
                         out + f->out_gen);
        f->out_gen += ch;
        input_index += 1.0 / src_ratio;
        rem = src_fmod_one(input_index);
        f->b_current = (f->b_current + ch * (int)lrint(input_index - rem)) % f->b_len;
        input_index = rem;
    }
    s->last_position = input_index;
    s->last_ratio = src_ratio;
    *in_used_frames = f->in_used / ch;
    *out_gen_frames = f->out_gen / ch;
    return 0;
}
