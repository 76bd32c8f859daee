// abi_biquad.cpp -- C ABI of the batched biquad: BiquadD::design + Biquad::new/apply
// (reference src/filter/biquad.rs:25-56, 73-155), Identity (src/filter/simple.rs:3-19), driven
// as Signal::filter (src/signal/mod.rs:42-48) on nch independent channels.  State (x1, x2,
// y1, y2 per channel) carries across calls; clone copies it (#[derive(Clone)], biquad.rs:4).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "abi_common.hpp"
#include "biquad_kernels.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

struct sdrgpu_biquad {
    int device = 0, sk = SDRGPU_F32, ident = 0;
    size_t nch = 1;
    float c[5] = {1.f, 0.f, 0.f, 0.f, 0.f};
    BiquadState* d_state = nullptr;
    StreamSlot stream;
    DevBuf stage_in, stage_out;
    // time-parallel blocks (biquad.hip): tp_seg / tp_warm 0 = automatic, tp_seg < 0 = serial
    long tp_seg = 0, tp_warm = 0;
    long simds = 1024;
    DevBuf spec_buf;
    long last_nseg = 0, last_nck = 0;

    // Warm-up for two trajectories of this recurrence to agree bit for bit: the slower pole of
    // 1 - na1 z^-1 - na2 z^-2 decays by r per sample, so 48 / -log2(r) samples shrink a start
    // difference by 2^-48 -- but the last ulps of difference random-walk under rounding before
    // they vanish (measured: the PLL's lock LowPass(20 kHz) at 1.8 Msps missed 2/3 of its
    // guesses after 48 / -log2(r) = 672 samples, none after 4 Ki), so the warm-up is 160 /
    // -log2(r) samples; above 64 Ki (poles within ~0.2 % of the unit circle, e.g. the stereo
    // pilot's LowPass(20 Hz) at 144 kHz, whose trajectories had not met after 220 Ki samples)
    // or for a pole on / outside the unit circle, 0 = no automatic time-parallel plan.
    // (profiles/r05_biquad_tp.jsonl)
    long auto_warm() const {
        const double a1 = c[3], a2 = c[4], disc = a1 * a1 + 4.0 * a2;
        double r;
        if (disc >= 0) {
            const double q = std::sqrt(disc);
            r = std::fmax(std::fabs(0.5 * (a1 + q)), std::fabs(0.5 * (a1 - q)));
        } else {
            r = std::sqrt(-a2);  // a complex pair: |z|^2 = -na2
        }
        if (!(r < 1.0)) return 0;
        const double w = r <= 0.0 ? 64.0 : std::ceil(160.0 / -std::log2(r));
        if (w > 65536.0) return 0;
        return std::max(((long)w + 7) / 8 * 8, 64L);
    }
    // The plan for a block of n samples: segments (0 = one serial pass) and warm-up.  Auto:
    // enough segments per channel to give every SIMD one wave (64 channel-segments each), none
    // shorter than 4 warm-ups or 4 Ki samples.
    void plan(long n, long* seg, long* warm) const {
        *seg = 0;
        const long aw = auto_warm();
        *warm = tp_warm > 0 ? (tp_warm + 7) / 8 * 8 : aw;
        if (ident || tp_seg < 0 || n <= 0 || (tp_seg == 0 && aw == 0)) return;
        long sg;
        if (tp_seg > 0) {
            sg = (tp_seg + 7) / 8 * 8;
        } else {
            const long minseg = std::max(4 * *warm, 4096L);
            const long by_lanes = 64 * simds / (long)nch, by_len = n / minseg;
            const long nseg = by_lanes < by_len ? by_lanes : by_len;
            if (nseg < 2) return;
            sg = ((n + nseg - 1) / nseg + 7) / 8 * 8;
        }
        if (n > sg) *seg = sg;
    }
    int make_spec(long n, BqSpec* sp, bool serial = false) {
        plan(n, &sp->seg, &sp->warm);
        last_nseg = 0;
        if (serial) sp->seg = 0;
        if (sp->seg <= 0) return SDRGPU_OK;
        sp->nseg = (n + sp->seg - 1) / sp->seg;
        long ck = sp->seg;  // checkpoints: at most 16 per segment, ck a multiple of 8 dividing seg
        for (long d = 16; d >= 2; --d)
            if (sp->seg % (8 * d) == 0 && sp->seg / d >= 512) { ck = sp->seg / d; break; }
        sp->ck = ck;
        const size_t nck = (size_t)(sp->seg / ck - 1);
        const size_t nstate = (size_t)sp->nseg * nch;
        // guess, end, end2, checkpoints, the counter (at state index (3 + nck) nstate), the marks
        const size_t bytes = (3 + nck) * nstate * sizeof(BiquadState) + 64 + nstate * sizeof(int);
        if (bytes > spec_buf.cap) {  // growing frees a buffer an earlier block may still use
            SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
            int st = spec_buf.ensure(bytes);
            if (st) return st;
        }
        sp->guess = static_cast<BiquadState*>(spec_buf.ptr);
        sp->end = sp->guess + nstate;
        sp->end2 = sp->end + nstate;
        sp->ckpt = nck ? sp->end2 + nstate : nullptr;
        sp->recomputed = reinterpret_cast<unsigned long long*>(sp->end2 + nstate + nck * nstate);
        sp->rstop = reinterpret_cast<int*>(sp->recomputed + 8);
        last_nseg = sp->nseg;
        last_nck = (long)nck;
        return SDRGPU_OK;
    }

    size_t sbytes() const { return kind_bytes(sk); }
    void free_all() {
        DeviceGuard g(device);
        if (d_state) (void)hipFree(d_state);
        d_state = nullptr;
        stage_in.release();
        stage_out.release();
        spec_buf.release();
        stream.destroy();
    }
    int reset() {
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_ERR_DEVICE;
        SDRGPU_HIP_TRY(hipMemsetAsync(d_state, 0, nch * sizeof(BiquadState), stream.cur));
        SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
        return SDRGPU_OK;
    }
    int init(int dev, int kind, const float* coefs, int identity, size_t channels) {
        if (!(kind == SDRGPU_F32 || kind == SDRGPU_C64) || channels == 0) return SDRGPU_ERR_INVALID;
        if (channels > (1u << 24)) return SDRGPU_ERR_UNSUPPORTED;
        int st = check_device(dev);
        if (st) return st;
        device = dev;
        sk = kind;
        nch = channels;
        ident = identity;
        std::memcpy(c, coefs, sizeof(c));
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_ERR_DEVICE;
        if ((st = stream.create())) return st;
        SDRGPU_HIP_TRY(hipMalloc(&d_state, nch * sizeof(BiquadState)));
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            simds = 4L * cus;
        return reset();
    }
    int run_dev(const void* in, size_t ld_in, size_t n, void* out, size_t ld_out) {
        if (n == 0) return SDRGPU_OK;
        if (!in || !out || ld_in < n || ld_out < n) return SDRGPU_ERR_INVALID;
        BqSpec sp;
        const size_t sb = sbytes();
        const bool alias = bytes_overlap(in, rows_span(nch, ld_in, n, sb), out, rows_span(nch, ld_out, n, sb));
        int st = make_spec((long)n, &sp, alias);
        if (st) return st;
        if (sp.seg > 0)
            return biquad_tp_launch(sk == SDRGPU_C64, (long)nch, c, in, (long)ld_in, (long)n, out,
                                    (long)ld_out, d_state, sp, stream.cur);
        return biquad_launch(sk == SDRGPU_C64, (long)nch, c, ident, in, (long)ld_in, (long)n, out,
                             (long)ld_out, d_state, stream.cur);
    }
};

extern "C" {

int sdrgpu_biquad_create(int device, int sample_kind, const sdrgpu_biquad_design* d, float rate,
                         size_t nch, sdrgpu_biquad** out) {
    if (!out || !d) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    float c[5];
    int ident = 0;
    int st = bq_design(*d, rate, c, &ident);
    if (st) return st;
    auto* h = new (std::nothrow) sdrgpu_biquad();
    if (!h) return SDRGPU_ERR_NOMEM;
    if ((st = h->init(device, sample_kind, c, ident, nch))) {
        h->free_all();
        delete h;
        return st;
    }
    *out = h;
    return SDRGPU_OK;
}

int sdrgpu_biquad_coefs(const sdrgpu_biquad* h, float* coefs5) {
    if (!h || !coefs5) return SDRGPU_ERR_INVALID;
    std::memcpy(coefs5, h->c, sizeof(h->c));
    return SDRGPU_OK;
}

int sdrgpu_biquad_set_stream(sdrgpu_biquad* h, void* s) {
    if (!h) return SDRGPU_ERR_INVALID;
    h->stream.set(s);
    return SDRGPU_OK;
}

int sdrgpu_biquad_get_stream(const sdrgpu_biquad* h, void** s) {
    if (!h || !s) return SDRGPU_ERR_INVALID;
    *s = h->stream.cur;
    return SDRGPU_OK;
}

int sdrgpu_biquad_process(sdrgpu_biquad* h, const void* in, size_t ld_in, size_t n, void* out,
                          size_t ld_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (n == 0) return SDRGPU_OK;
    if (!in || !out || ld_in < n || ld_out < n) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const size_t sb = h->sbytes(), nch = h->nch;
    int st;
    if ((st = h->stage_in.ensure(nch * n * sb))) return st;
    if ((st = h->stage_out.ensure(nch * n * sb))) return st;
    SDRGPU_HIP_TRY(hipMemcpy2DAsync(h->stage_in.ptr, n * sb, in, ld_in * sb, n * sb, nch,
                                    hipMemcpyHostToDevice, h->stream.cur));
    if ((st = h->run_dev(h->stage_in.ptr, n, n, h->stage_out.ptr, n))) return st;
    SDRGPU_HIP_TRY(hipMemcpy2DAsync(out, ld_out * sb, h->stage_out.ptr, n * sb, n * sb, nch,
                                    hipMemcpyDeviceToHost, h->stream.cur));
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_biquad_process_dev(sdrgpu_biquad* h, const void* d_in, size_t ld_in, size_t n,
                              void* d_out, size_t ld_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    return h->run_dev(d_in, ld_in, n, d_out, ld_out);
}

int sdrgpu_biquad_set_time_parallel(sdrgpu_biquad* h, long seg, long warm) {
    if (!h || warm < 0) return SDRGPU_ERR_INVALID;
    h->tp_seg = seg;
    h->tp_warm = warm;
    return SDRGPU_OK;
}

int sdrgpu_biquad_time_parallel_plan(const sdrgpu_biquad* h, size_t n, long* seg, long* warm) {
    if (!h || !seg || !warm) return SDRGPU_ERR_INVALID;
    h->plan((long)n, seg, warm);
    return SDRGPU_OK;
}

int sdrgpu_biquad_last_time_parallel(sdrgpu_biquad* h, long* segments, long* recomputed) {
    if (!h || !segments || !recomputed) return SDRGPU_ERR_INVALID;
    *segments = h->last_nseg;
    *recomputed = 0;
    if (h->last_nseg > 0) {
        DeviceGuard g(h->device);
        unsigned long long r = 0;
        const auto* base = static_cast<const BiquadState*>(h->spec_buf.ptr);
        SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
        SDRGPU_HIP_TRY(hipMemcpy(&r, base + (3 + h->last_nck) * h->last_nseg * (long)h->nch, sizeof(r),
                                 hipMemcpyDeviceToHost));
        *recomputed = (long)r;
    }
    return SDRGPU_OK;
}

int sdrgpu_biquad_sync(sdrgpu_biquad* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_biquad_reset(sdrgpu_biquad* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    return h->reset();
}

int sdrgpu_biquad_clone(const sdrgpu_biquad* h, sdrgpu_biquad** out) {
    if (!h || !out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    auto* c = new (std::nothrow) sdrgpu_biquad();
    if (!c) return SDRGPU_ERR_NOMEM;
    int st = c->init(h->device, h->sk, h->c, h->ident, h->nch);
    c->tp_seg = h->tp_seg;
    c->tp_warm = h->tp_warm;
    if (!st) {
        DeviceGuard g(h->device);
        if (hipMemcpyAsync(c->d_state, h->d_state, h->nch * sizeof(BiquadState),
                           hipMemcpyDeviceToDevice, h->stream.cur) != hipSuccess ||
            hipStreamSynchronize(h->stream.cur) != hipSuccess)
            st = SDRGPU_ERR_DEVICE;
    }
    if (st) {
        c->free_all();
        delete c;
        return st;
    }
    *out = c;
    return SDRGPU_OK;
}

void sdrgpu_biquad_destroy(sdrgpu_biquad* h) {
    if (!h) return;
    h->free_all();
    delete h;
}

}  // extern "C"
