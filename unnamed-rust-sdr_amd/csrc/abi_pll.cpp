// abi_pll.cpp -- C ABI of the batched PLL: PllDesign::new/design (reference
// src/filter/pll.rs:25-60) with BiquadD designs (src/filter/biquad.rs:73-155) or Identity.
#include <cmath>
#include <cstring>
#include <vector>

#include "abi_common.hpp"
#include "pll_kernels.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

namespace {

// Biquad::new normalisation (biquad.rs:25-38)
void bq_new(float a0, float a1, float a2, float b0, float b1, float b2, float* c) {
    c[0] = b0 / a0;
    c[1] = b1 / a0;
    c[2] = b2 / a0;
    c[3] = -a1 / a0;
    c[4] = -a2 / a0;
}

}  // namespace

// BiquadD::design (biquad.rs:83-155), host f32 math (glibc libm like Rust std); shared with
// the standalone biquad ABI (abi_biquad.cpp).  This file is built with -ffp-contract=off.
int sdrgpu::detail::bq_design(const sdrgpu_biquad_design& d, float rate, float* c, int* ident) {
    const float PI = 3.14159265358979323846f;
    *ident = 0;
    float omega, cs, alpha;
    switch (d.kind) {
    case SDRGPU_BQ_IDENTITY:
        *ident = 1;
        c[0] = 1.f; c[1] = c[2] = c[3] = c[4] = 0.f;
        return SDRGPU_OK;
    case SDRGPU_BQ_LOWPASS:
        omega = 2.0f * PI * d.freq / rate; cs = cosf(omega); alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, (1.0f - cs) / 2.0f, 1.0f - cs, (1.0f - cs) / 2.0f, c);
        return SDRGPU_OK;
    case SDRGPU_BQ_HIGHPASS:
        omega = 2.0f * PI * d.freq / rate; cs = cosf(omega); alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, (1.0f + cs) / 2.0f, -1.0f - cs, (1.0f + cs) / 2.0f, c);
        return SDRGPU_OK;
    case SDRGPU_BQ_BANDPASS:
        omega = 2.0f * PI * d.freq / rate; cs = cosf(omega); alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, alpha, 0.0f, -alpha, c);
        return SDRGPU_OK;
    case SDRGPU_BQ_NOTCH:
        omega = 2.0f * PI * d.freq / rate; cs = cosf(omega); alpha = sinf(omega) / (2.0f * d.q);
        bq_new(1.0f + alpha, -2.0f * cs, 1.0f - alpha, 1.0f, -2.0f * cs, 1.0f, c);
        return SDRGPU_OK;
    case SDRGPU_BQ_LR: {
        const float decayn = d.freq / rate;
        bq_new(1.0f, -expf(-decayn), 0.0f, decayn, 0.0f, 0.0f, c);
        return SDRGPU_OK;
    }
    default:
        return SDRGPU_ERR_INVALID;
    }
}


struct sdrgpu_pll {
    int device = 0;
    sdrgpu_pll_params params{};
    PllDevParams dp{};
    PllChannelState* d_state = nullptr;
    StreamSlot stream;
    DevBuf stage_in, stage_out, stage_lock;
    AsyncD2H async;
    // time-parallel segments (pll.hip): requested segment / warm-up lengths (0 = auto, segment
    // < 0 = always one serial pass), the device's SIMD count, and the [2][segments][nch] states
    long tp_seg = 0, tp_warm = 0;
    long simds = 1024;
    DevBuf spec_buf;
    long last_nseg = 0;  // segments of the most recent time-parallel block (0: serial)
    long last_nck = 0;   // and the checkpoints per segment it kept
    // Automatic plan, adapted per handle: when most segments of a time-parallel block had to be
    // recomputed (an unlocked loop on noise: trajectories that never meet bit for bit), the next
    // kSerialBlocks blocks run one serial pass and the handle then probes again.  The recompute
    // count of each automatic time-parallel block is copied to pinned memory behind an event,
    // and read by a later block's plan only once the event has completed (no stream sync).
    static constexpr int kSerialBlocks = 8;
    hipEvent_t probe_ev = nullptr;
    unsigned long long* probe_host = nullptr;
    bool probe_pending = false;
    long probe_total = 0;
    int serial_left = 0;
    // sdrgpu_pll_set_phase_timing: events around the three kernels of a time-parallel block
    hipEvent_t phase_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool phase_on = false;

    bool adapt_serial() {
        if (tp_seg != 0) return false;
        if (probe_pending && hipEventQuery(probe_ev) == hipSuccess) {
            probe_pending = false;
            if (2 * (long)*probe_host > probe_total) serial_left = kSerialBlocks;
        }
        if (serial_left > 0) {
            --serial_left;
            return true;
        }
        return false;
    }
    // after a launch: record this block's recompute count for the next plans
    int probe(const PllSpec& sp) {
        if (tp_seg != 0 || sp.seg <= 0 || probe_pending || !probe_ev) return SDRGPU_OK;
        SDRGPU_HIP_TRY(hipMemcpyAsync(probe_host, sp.recomputed, sizeof(*probe_host), hipMemcpyDeviceToHost,
                                      stream.cur));
        SDRGPU_HIP_TRY(hipEventRecord(probe_ev, stream.cur));
        probe_pending = true;
        probe_total = last_nseg * dp.nch;
        return SDRGPU_OK;
    }

    // The plan for a block of n samples.  Auto: enough segments per channel to give every SIMD
    // one wave (64 channel-segments each), none shorter than 4 Ki samples, warm-up 4 Ki.  A
    // segment's pass-1 trajectory has had warm-up + segment samples to meet the true one before
    // its successor's re-run starts from its end; every configs[3] channel's state had converged
    // within 12.2 Ki.  Measured: configs[3] (64 segments of 16 Ki either way)
    // 8 Ki to 16 Ki of warm-up all at 11.4-13.2 ms (profiles/r05_pll_refix_sweep.txt); one
    // 1.8 Msps stream in main.rs's 0.1 s blocks, 4 Ki segments 6.2 ms per block against 9.7 at
    // the 16 Ki minimum and 53 serially, 2 Ki segments 20 ms (profiles/r05_pll_tp_single.txt).
    static constexpr long kMinSeg = 4096, kWarm = 4096;
    void plan(long n, long* seg, long* warm) const {
        *seg = 0;
        *warm = tp_warm > 0 ? (tp_warm + 7) / 8 * 8 : kWarm;
        if (tp_seg < 0 || n <= 0) return;
        long sg;
        if (tp_seg > 0) {
            sg = (tp_seg + 7) / 8 * 8;
        } else {
            const long by_lanes = 64 * simds / dp.nch, by_len = n / kMinSeg;
            const long nseg = by_lanes < by_len ? by_lanes : by_len;
            if (nseg < 2) return;
            sg = ((n + nseg - 1) / nseg + 7) / 8 * 8;
        }
        if (n > sg) *seg = sg;
    }

    int make_spec(long n, PllSpec* sp, bool serial = false) {
        plan(n, &sp->seg, &sp->warm);
        last_nseg = 0;
        if (sp->seg > 0 && adapt_serial()) serial = true;
        if (serial) sp->seg = 0;
        if (sp->seg <= 0) return SDRGPU_OK;
        const long nseg = (n + sp->seg - 1) / sp->seg;
        // checkpoints every ck samples: at most 16 per segment, ck a multiple of 8 dividing seg
        long ck = sp->seg;
        for (long d = 16; d >= 2; --d)
            if (sp->seg % (8 * d) == 0 && sp->seg / d >= 1024) { ck = sp->seg / d; break; }
        sp->ck = ck;
        const size_t nck = (size_t)(sp->seg / ck - 1);
        const size_t nstate = (size_t)nseg * (size_t)dp.nch;
        // guess, end, end2, checkpoints, the counter (sdrgpu_pll_last_time_parallel reads it at
        // state index (3 + nck) nstate), then the re-run marks
        const size_t bytes = (3 + nck) * nstate * sizeof(PllChannelState) + nstate * sizeof(int) + 64;
        if (bytes > spec_buf.cap) {  // growing frees a buffer an earlier block may still use
            SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
            int st = spec_buf.ensure(bytes);
            if (st) return st;
        }
        sp->guess = static_cast<PllChannelState*>(spec_buf.ptr);
        sp->end = sp->guess + nseg * dp.nch;
        sp->end2 = sp->end + nstate;
        sp->ckpt = nck ? sp->end2 + nstate : nullptr;
        sp->recomputed = reinterpret_cast<unsigned long long*>(sp->end2 + nstate + nck * nstate);
        sp->rstop = reinterpret_cast<int*>(sp->recomputed + 8);
        sp->phase_ev = phase_on ? phase_ev : nullptr;
        last_nseg = nseg;
        last_nck = (long)nck;
        return SDRGPU_OK;
    }

    void free_all() {
        DeviceGuard g(device);
        if (d_state) (void)hipFree(d_state);
        d_state = nullptr;
        if (probe_ev) (void)hipEventDestroy(probe_ev);
        probe_ev = nullptr;
        for (auto& e : phase_ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        if (probe_host) (void)hipHostFree(probe_host);
        probe_host = nullptr;
        async.release();
        stage_in.release();
        stage_out.release();
        stage_lock.release();
        spec_buf.release();
        stream.destroy();
    }
};

extern "C" {

int sdrgpu_pll_reset(sdrgpu_pll* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    // PllDesign::design: nphase = 0, value = 0 + 0i, filter states zero (pll.rs:57-58)
    SDRGPU_HIP_TRY(hipMemsetAsync(h->d_state, 0, h->dp.nch * sizeof(PllChannelState), h->stream.cur));
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    h->probe_pending = false;  // the adapted plan starts over with the stream
    h->serial_left = 0;
    return SDRGPU_OK;
}

int sdrgpu_pll_create(int device, const sdrgpu_pll_params* p, size_t nch, sdrgpu_pll** out) {
    if (!out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    if (!p || nch == 0 || !(p->rate > 0.0f)) return SDRGPU_ERR_INVALID;
    int st = check_device(device);
    if (st) return st;
    auto* h = new (std::nothrow) sdrgpu_pll();
    if (!h) return SDRGPU_ERR_NOMEM;
    h->device = device;
    h->params = *p;
    PllDevParams& d = h->dp;
    d.nch = (long)nch;
    d.rate = p->rate;
    d.reference = p->reference / p->rate;  // pll.rs:51
    d.gain = p->gain;
    if ((st = bq_design(p->loopf, p->rate, d.loopc, &d.loop_ident)) ||
        (st = bq_design(p->outputf, p->rate, d.outc, &d.out_ident)) ||
        (st = bq_design(p->lockf, p->rate, d.lockc, &d.lock_ident))) {
        delete h;
        return st;
    }
    {
        DeviceGuard g(device);
        if (!g.ok()) st = SDRGPU_ERR_DEVICE;
        if (!st) st = h->stream.create();
        if (!st && hipMalloc(&h->d_state, nch * sizeof(PllChannelState)) != hipSuccess) st = SDRGPU_ERR_NOMEM;
        if (!st && (hipHostMalloc(reinterpret_cast<void**>(&h->probe_host), sizeof(*h->probe_host)) != hipSuccess ||
                    hipEventCreateWithFlags(&h->probe_ev, hipEventDisableTiming) != hipSuccess))
            st = SDRGPU_ERR_NOMEM;
        int cus = 0;
        if (!st && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
            cus > 0)
            h->simds = 4L * cus;
    }
    if (!st) st = sdrgpu_pll_reset(h);
    if (st) {
        h->free_all();
        delete h;
        return st;
    }
    *out = h;
    return SDRGPU_OK;
}

int sdrgpu_pll_set_input_kind(sdrgpu_pll* h, int sample_kind) {
    if (!h || (sample_kind != SDRGPU_C64 && sample_kind != SDRGPU_CU8)) return SDRGPU_ERR_INVALID;
    h->dp.in_u8 = sample_kind == SDRGPU_CU8;
    return SDRGPU_OK;
}

int sdrgpu_pll_set_output_mode(sdrgpu_pll* h, int mode) {
    if (!h || mode < SDRGPU_PLL_OUT_FILTER || mode > SDRGPU_PLL_OUT_STEREO_DIFF)
        return SDRGPU_ERR_INVALID;
    h->dp.out_mode = mode;
    return SDRGPU_OK;
}

int sdrgpu_pll_set_time_parallel(sdrgpu_pll* h, long seg, long warm) {
    if (!h || warm < 0) return SDRGPU_ERR_INVALID;
    h->tp_seg = seg;
    h->tp_warm = warm;
    return SDRGPU_OK;
}

int sdrgpu_pll_time_parallel_plan(const sdrgpu_pll* h, size_t n, long* seg, long* warm) {
    if (!h || !seg || !warm) return SDRGPU_ERR_INVALID;
    h->plan((long)n, seg, warm);
    return SDRGPU_OK;
}

int sdrgpu_pll_last_time_parallel(sdrgpu_pll* h, long* segments, long* recomputed) {
    if (!h || !segments || !recomputed) return SDRGPU_ERR_INVALID;
    *segments = h->last_nseg;
    *recomputed = 0;
    if (h->last_nseg > 0) {
        DeviceGuard g(h->device);
        unsigned long long r = 0;
        const auto* base = static_cast<const PllChannelState*>(h->spec_buf.ptr);
        SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
        SDRGPU_HIP_TRY(hipMemcpy(&r, base + (3 + h->last_nck) * h->last_nseg * h->dp.nch, sizeof(r),
                                 hipMemcpyDeviceToHost));
        *recomputed = (long)r;
    }
    return SDRGPU_OK;
}

int sdrgpu_pll_set_phase_timing(sdrgpu_pll* h, int on) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (on && !h->phase_ev[0])
        for (auto& e : h->phase_ev) SDRGPU_HIP_TRY(hipEventCreate(&e));
    h->phase_on = on != 0;
    return SDRGPU_OK;
}

int sdrgpu_pll_last_phase_ms(sdrgpu_pll* h, float* pass1, float* rerun, float* walk) {
    if (!h || !pass1 || !rerun || !walk) return SDRGPU_ERR_INVALID;
    *pass1 = *rerun = *walk = 0.f;
    if (!h->phase_on || h->last_nseg <= 0) return SDRGPU_OK;
    DeviceGuard g(h->device);
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    SDRGPU_HIP_TRY(hipEventElapsedTime(pass1, h->phase_ev[0], h->phase_ev[1]));
    SDRGPU_HIP_TRY(hipEventElapsedTime(rerun, h->phase_ev[1], h->phase_ev[2]));
    SDRGPU_HIP_TRY(hipEventElapsedTime(walk, h->phase_ev[2], h->phase_ev[3]));
    return SDRGPU_OK;
}

int sdrgpu_pll_set_stream(sdrgpu_pll* h, void* s) {
    if (!h) return SDRGPU_ERR_INVALID;
    h->stream.set(s);
    return SDRGPU_OK;
}

int sdrgpu_pll_get_stream(const sdrgpu_pll* h, void** s) {
    if (!h || !s) return SDRGPU_ERR_INVALID;
    *s = h->stream.cur;
    return SDRGPU_OK;
}

int sdrgpu_pll_process_dev(sdrgpu_pll* h, const void* d_in, size_t ld_in, size_t n, float* d_out,
                           uint8_t* d_locked, size_t ld_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (n == 0) return SDRGPU_OK;
    if (!d_in || !d_out || !d_locked || ld_in < n || ld_out < n) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    // an output range overlapping the input takes the serial pass (bytes_overlap, abi_common.hpp)
    const size_t nch = (size_t)h->dp.nch, in_bytes = rows_span(nch, ld_in, n, h->dp.in_u8 ? 2 : sizeof(float2));
    const bool alias = bytes_overlap(d_in, in_bytes, d_out, rows_span(nch, ld_out, n, sizeof(float))) ||
                       bytes_overlap(d_in, in_bytes, d_locked, rows_span(nch, ld_out, n, 1));
    PllSpec sp;
    int st = h->make_spec((long)n, &sp, alias);
    if (st) return st;
    if ((st = pll_launch(h->dp, d_in, (long)ld_in, (long)n, d_out, d_locked, (long)ld_out, h->d_state, sp,
                         h->stream.cur)))
        return st;
    return h->probe(sp);
}

int sdrgpu_pll_process(sdrgpu_pll* h, const void* in, size_t ld_in, size_t n, float* out,
                       uint8_t* locked, size_t ld_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (n == 0) return SDRGPU_OK;
    if (!in || !out || !locked || ld_in < n || ld_out < n) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const size_t nch = (size_t)h->dp.nch;
    int st;
    const size_t sb = h->dp.in_u8 ? 2 : sizeof(float2);  // bytes per input sample
    if ((st = h->stage_in.ensure(nch * n * sb)) ||
        (st = h->stage_out.ensure(nch * n * sizeof(float))) ||
        (st = h->stage_lock.ensure(nch * n)))
        return st;
    PllSpec sp;
    if ((st = h->make_spec((long)n, &sp))) return st;
    SDRGPU_HIP_TRY(hipMemcpy2DAsync(h->stage_in.ptr, n * sb, in, ld_in * sb, n * sb, nch,
                                    hipMemcpyHostToDevice, h->stream.cur));
    if ((st = pll_launch(h->dp, h->stage_in.ptr, (long)n, (long)n,
                         static_cast<float*>(h->stage_out.ptr), static_cast<uint8_t*>(h->stage_lock.ptr),
                         (long)n, h->d_state, sp, h->stream.cur)) || (st = h->probe(sp)))
        return st;
    SDRGPU_HIP_TRY(hipMemcpy2DAsync(out, ld_out * sizeof(float), h->stage_out.ptr, n * sizeof(float),
                                    n * sizeof(float), nch, hipMemcpyDeviceToHost, h->stream.cur));
    SDRGPU_HIP_TRY(hipMemcpy2DAsync(locked, ld_out, h->stage_lock.ptr, n, n, nch, hipMemcpyDeviceToHost,
                                    h->stream.cur));
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_pll_process_async(sdrgpu_pll* h, const void* in, size_t n, float* out,
                             uint8_t* locked) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (n == 0) return SDRGPU_OK;
    if (!in || !out || !locked) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const size_t nch = (size_t)h->dp.nch;
    const size_t sb = h->dp.in_u8 ? 2 : sizeof(float2);
    int st, slot = 0;
    if (h->stage_in.cap < nch * n * sb) {  // growing frees a buffer an earlier block may read
        SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
        if ((st = h->stage_in.ensure(nch * n * sb))) return st;
    }
    const size_t ob[2] = {nch * n * sizeof(float), nch * n};
    if ((st = h->async.acquire(h->stream.cur, ob, 2, &slot))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(h->stage_in.ptr, in, nch * n * sb, hipMemcpyHostToDevice,
                                  h->stream.cur));
    float* d_out = static_cast<float*>(h->async.out[slot][0].ptr);
    uint8_t* d_lock = static_cast<uint8_t*>(h->async.out[slot][1].ptr);
    PllSpec sp;
    if ((st = h->make_spec((long)n, &sp))) return st;
    if ((st = pll_launch(h->dp, h->stage_in.ptr, (long)n, (long)n, d_out, d_lock, (long)n,
                         h->d_state, sp, h->stream.cur)) || (st = h->probe(sp)))
        return st;
    if ((st = h->async.begin_download(h->stream.cur, slot))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(out, d_out, ob[0], hipMemcpyDeviceToHost, h->async.d2h));
    SDRGPU_HIP_TRY(hipMemcpyAsync(locked, d_lock, ob[1], hipMemcpyDeviceToHost, h->async.d2h));
    return h->async.end_download(slot);
}

int sdrgpu_pll_state(sdrgpu_pll* h, size_t ch, float* nphase, float* value_re_im) {
    if (!h || (long)ch >= h->dp.nch) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    PllChannelState s;
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    SDRGPU_HIP_TRY(hipMemcpy(&s, h->d_state + ch, sizeof(s), hipMemcpyDeviceToHost));
    if (nphase) *nphase = s.nphase;
    if (value_re_im) {
        value_re_im[0] = s.vr;
        value_re_im[1] = s.vi;
    }
    return SDRGPU_OK;
}

int sdrgpu_pll_sync(sdrgpu_pll* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return h->async.sync();
}

int sdrgpu_pll_clone(const sdrgpu_pll* h, sdrgpu_pll** out) {
    if (!h || !out) return SDRGPU_ERR_INVALID;
    int st = sdrgpu_pll_create(h->device, &h->params, (size_t)h->dp.nch, out);
    if (st) return st;
    (*out)->dp.out_mode = h->dp.out_mode;
    (*out)->dp.in_u8 = h->dp.in_u8;
    (*out)->tp_seg = h->tp_seg;
    (*out)->tp_warm = h->tp_warm;
    DeviceGuard g(h->device);
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    SDRGPU_HIP_TRY(hipMemcpy((*out)->d_state, h->d_state, h->dp.nch * sizeof(PllChannelState),
                             hipMemcpyDeviceToDevice));
    return SDRGPU_OK;
}

int sdrgpu_debug_libm(int device, int fn, const float* a, const float* b, float* out0,
                      float* out1, size_t n) {
    if ((fn != SDRGPU_DEBUG_ATAN2F && fn != SDRGPU_DEBUG_SINCOSF) || (n && (!a || !out0)) ||
        (n && fn == SDRGPU_DEBUG_ATAN2F && !b) || (n && fn == SDRGPU_DEBUG_SINCOSF && !out1))
        return SDRGPU_ERR_INVALID;
    if (int st = check_device(device)) return st;
    if (n == 0) return SDRGPU_OK;
    DeviceGuard g(device);
    DevBuf da, db, d0, d1;
    const size_t bytes = n * sizeof(float);
    int st = da.ensure(bytes);
    if (!st) st = d0.ensure(bytes);
    if (!st && fn == SDRGPU_DEBUG_ATAN2F) st = db.ensure(bytes);
    if (!st && fn == SDRGPU_DEBUG_SINCOSF) st = d1.ensure(bytes);
    if (!st && hipMemcpy(da.ptr, a, bytes, hipMemcpyHostToDevice) != hipSuccess) st = SDRGPU_ERR_DEVICE;
    if (!st && db.ptr && hipMemcpy(db.ptr, b, bytes, hipMemcpyHostToDevice) != hipSuccess)
        st = SDRGPU_ERR_DEVICE;
    if (!st)
        st = libm_debug_launch(fn, (const float*)da.ptr, (const float*)db.ptr, (float*)d0.ptr,
                               (float*)d1.ptr, (long)n, nullptr);
    if (!st && hipDeviceSynchronize() != hipSuccess) st = SDRGPU_ERR_DEVICE;
    if (!st && hipMemcpy(out0, d0.ptr, bytes, hipMemcpyDeviceToHost) != hipSuccess) st = SDRGPU_ERR_DEVICE;
    if (!st && d1.ptr && hipMemcpy(out1, d1.ptr, bytes, hipMemcpyDeviceToHost) != hipSuccess)
        st = SDRGPU_ERR_DEVICE;
    da.release();
    db.release();
    d0.release();
    d1.release();
    return st;
}

void sdrgpu_pll_destroy(sdrgpu_pll* h) {
    if (!h) return;
    h->free_all();
    delete h;
}

}  // extern "C"
