// abi_fir.cpp -- C ABI of the streaming FIR / FIR-decimate and the FIR bank.
//
// Replaces Fir::new/apply + FilterDesign (reference src/filter/fir.rs:12-58) driven by
// adapters::Filter (src/signal/adapters/mod.rs:77-96) and Decimate
// (src/signal/adapters/mod.rs:19-37).  Stream state (K-1 history per channel, decimation
// phase) is carried across calls so block partitioning never changes the outputs.
#include <vector>

#include "abi_common.hpp"
#include "fir_kernels.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

namespace sdrgpu {
int fir_os_launch(const FirParams& p, void* os_state, hipStream_t s);
void* fir_os_prepare(int device, int sample_kind, int tap_kind, const void* taps, int K,
                     int D, hipStream_t s, int* status);
void fir_os_release(void* os_state);
int fir_mx_supported(int sample_kind, int tap_kind, int K, int D);
void* fir_mx_prepare(int device, const float* taps, int K, int D, int* status);
int fir_mx_launch(const FirParams& p, void* state, hipStream_t s, int* kernel);
void fir_mx_release(void* state);
int cu8_to_c64_launch(const void* in, long ld_in, long n, long nch, void* out, hipStream_t s);
}  // namespace sdrgpu

struct FirCore {
    int device = 0;
    int sk = SDRGPU_C64, tk = SDRGPU_F32;
    int csk = SDRGPU_C64;  // compute kind: CU8 input is filtered as C64
    int K = 1, D = 1;
    size_t nch = 1;
    int algo = SDRGPU_FIR_AUTO;
    int last_algo = SDRGPU_FIR_AUTO;       // path that ran the most recent block
    int last_kernel = SDRGPU_FIR_KERNEL_NONE;  // and its kernel (sdrgpu_fir_kernel)
    std::vector<unsigned char> taps_host;  // original taps (for clone / OS prep)
    int tpp = 0;
    void* d_taps_pm = nullptr;
    void* d_hist[2] = {nullptr, nullptr};  // ping-pong, nch x (K-1) samples each
    int cur = 0;
    unsigned long long seen = 0;           // stream samples consumed (decimation phase)
    StreamSlot stream;
    DevBuf stage_in, stage_out, stage_conv, stage_alias;
    void* os_state = nullptr;              // overlap-save plan (lazily built)
    int os_status = SDRGPU_OK;
    void* mx_state = nullptr;              // split-bf16 MFMA direct-form plan (lazily built)
    int mx_status = SDRGPU_OK;
    // async host streaming: downloads on their own stream (block i's D2H overlaps block
    // i+1's H2D -- PCIe is full duplex), two output slots guarded by events
    hipStream_t d2h = nullptr;
    hipEvent_t ev_k[2] = {nullptr, nullptr}, ev_o[2] = {nullptr, nullptr};
    bool ev_o_live[2] = {false, false};
    DevBuf stage_aout[2];
    int aslot = 0;

    size_t in_bytes() const { return kind_bytes(sk); }
    size_t out_bytes() const { return kind_bytes(csk); }
    size_t hist_bytes() const { return nch * (size_t)(K - 1) * out_bytes(); }

    long first_kept() const {
        const long g = (long)(seen % (unsigned long long)D);
        return ((long)D - 1 - g) % D;
    }
    size_t out_len(size_t n_in) const {
        const long i0 = first_kept();
        return (long)n_in > i0 ? (size_t)(((long)n_in - 1 - i0) / D + 1) : 0;
    }

    void free_all() {
        DeviceGuard g(device);
        if (d_taps_pm) (void)hipFree(d_taps_pm);
        for (auto& p : d_hist)
            if (p) (void)hipFree(p);
        d_taps_pm = nullptr;
        d_hist[0] = d_hist[1] = nullptr;
        stage_in.release();
        stage_out.release();
        stage_conv.release();
        stage_alias.release();
        if (os_state) fir_os_release(os_state);
        os_state = nullptr;
        if (mx_state) fir_mx_release(mx_state);
        mx_state = nullptr;
        if (d2h) (void)hipStreamSynchronize(d2h);
        for (int i = 0; i < 2; ++i) {
            stage_aout[i].release();
            if (ev_k[i]) (void)hipEventDestroy(ev_k[i]);
            if (ev_o[i]) (void)hipEventDestroy(ev_o[i]);
            ev_k[i] = ev_o[i] = nullptr;
            ev_o_live[i] = false;
        }
        if (d2h) (void)hipStreamDestroy(d2h);
        d2h = nullptr;
        stream.destroy();
    }
    int sync_all() {
        DeviceGuard g(device);
        SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
        if (d2h) SDRGPU_HIP_TRY(hipStreamSynchronize(d2h));
        return SDRGPU_OK;
    }

    int reset_state() {
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_ERR_DEVICE;
        seen = 0;
        cur = 0;
        if (K > 1) {
            SDRGPU_HIP_TRY(hipMemsetAsync(d_hist[0], 0, hist_bytes(), stream.cur));
            SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
        }
        return SDRGPU_OK;
    }

    int init(int dev, int sample_kind, int tap_kind, const void* taps, size_t ntaps,
             uint32_t decim, size_t channels) {
        if (!taps || ntaps == 0 || decim == 0 || channels == 0) return SDRGPU_ERR_INVALID;
        if (ntaps > (1u << 20) || decim > (1u << 20) || channels > (1u << 24))
            return SDRGPU_ERR_UNSUPPORTED;
        if (!((sample_kind == SDRGPU_F32 && tap_kind == SDRGPU_F32) ||
              (sample_kind == SDRGPU_C64 && tap_kind == SDRGPU_F32) ||
              (sample_kind == SDRGPU_C64 && tap_kind == SDRGPU_C64) ||
              (sample_kind == SDRGPU_CU8 && tap_kind == SDRGPU_F32) ||
              (sample_kind == SDRGPU_CU8 && tap_kind == SDRGPU_C64)))
            return SDRGPU_ERR_INVALID;
        int st = check_device(dev);
        if (st) return st;
        device = dev;
        sk = sample_kind;
        csk = sample_kind == SDRGPU_CU8 ? SDRGPU_C64 : sample_kind;
        tk = tap_kind;
        K = (int)ntaps;
        D = (int)decim;
        nch = channels;
        const size_t tb = kind_bytes(tk);
        taps_host.assign((const unsigned char*)taps, (const unsigned char*)taps + tb * ntaps);

        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_ERR_DEVICE;
        if ((st = stream.create())) return st;
        // polyphase-major padded taps: taps_pm[p*tpp + i] = h[p + i*D]
        tpp = taps_per_phase(K, D);
        std::vector<unsigned char> pm((size_t)D * tpp * tb, 0);
        for (int k = 0; k < K; ++k)
            std::memcpy(&pm[((size_t)(k % D) * tpp + k / D) * tb], &taps_host[(size_t)k * tb], tb);
        SDRGPU_HIP_TRY(hipMalloc(&d_taps_pm, pm.size()));
        SDRGPU_HIP_TRY(hipMemcpy(d_taps_pm, pm.data(), pm.size(), hipMemcpyHostToDevice));
        if (K > 1) {
            SDRGPU_HIP_TRY(hipMalloc(&d_hist[0], hist_bytes()));
            SDRGPU_HIP_TRY(hipMalloc(&d_hist[1], hist_bytes()));
        }
        return reset_state();
    }

    bool want_mx() const {
        if (algo != SDRGPU_FIR_AUTO && algo != SDRGPU_FIR_MATRIX) return false;
        return fir_mx_supported(csk, tk, K, D) != 0;
    }

    bool want_os() const {
        if (algo == SDRGPU_FIR_DIRECT || algo == SDRGPU_FIR_MATRIX) return false;
        if (!fir_os_supported(csk, tk, K, D)) return false;
        return true;  // AUTO or OVERLAP_SAVE
    }

    // Enqueue one block (device pointers) on the current stream.
    int run_dev(const void* d_in, size_t ld_in, size_t n_in, void* d_out, size_t ld_out,
                size_t* n_out_ret) {
        const size_t n_out = out_len(n_in);
        if (n_out_ret) *n_out_ret = n_out;
        if (n_in == 0) return SDRGPU_OK;
        if (!d_in || (n_out > 0 && !d_out)) return SDRGPU_ERR_INVALID;
        int st = unalias_input(stage_alias, d_in, rows_span(nch, ld_in, n_in, in_bytes()), d_out,
                               rows_span(nch, ld_out, n_out, out_bytes()), stream.cur);
        if (st) return st;
        FirParams p{};
        p.sample_kind = sk;
        p.tap_kind = tk;
        p.in = d_in;
        p.ld_in = (long)ld_in;
        p.n_in = (long)n_in;
        // K == 1 has no history: point both at a harmless non-null buffer.
        p.hist = K > 1 ? d_hist[cur] : d_taps_pm;
        p.hist_next = K > 1 ? d_hist[cur ^ 1] : nullptr;
        p.i0 = first_kept();
        p.n_out = (long)n_out;
        p.K = K;
        p.D = D;
        p.taps_pm = d_taps_pm;
        p.tpp = tpp;
        p.out = d_out;
        p.ld_out = (long)ld_out;
        p.nch = (int)nch;
        p.force_naive = 0;
        st = SDRGPU_ERR_UNSUPPORTED;
        int ran = SDRGPU_FIR_MATRIX;
        int kern = SDRGPU_FIR_KERNEL_NONE, conv = 0;
        if (want_mx()) {
            if (!mx_state && mx_status == SDRGPU_OK)
                mx_state = fir_mx_prepare(device, reinterpret_cast<const float*>(taps_host.data()),
                                          K, D, &mx_status);
            if (mx_state) st = fir_mx_launch(p, mx_state, stream.cur, &kern);  // CU8: fused ingest
            else if (mx_status != SDRGPU_ERR_UNSUPPORTED) return mx_status;
            // an unaligned buffer (UNSUPPORTED) falls through to the other paths
            if (st != SDRGPU_OK && st != SDRGPU_ERR_UNSUPPORTED) return st;
        }
        if (st != SDRGPU_OK && sk == SDRGPU_CU8) {
            // not fused for this shape: convert the block to C64 (RtlTcpSignal::next), then
            // filter it like any C64 block
            if ((st = stage_conv.ensure(nch * n_in * sizeof(float) * 2))) return st;
            if ((st = cu8_to_c64_launch(d_in, (long)ld_in, (long)n_in, (long)nch, stage_conv.ptr,
                                        stream.cur)))
                return st;
            p.sample_kind = SDRGPU_C64;
            p.in = stage_conv.ptr;
            p.ld_in = (long)n_in;
            conv = SDRGPU_FIR_KERNEL_CU8_CONVERTED;
            st = SDRGPU_ERR_UNSUPPORTED;
            if (want_mx() && mx_state) {
                st = fir_mx_launch(p, mx_state, stream.cur, &kern);
                if (st != SDRGPU_OK && st != SDRGPU_ERR_UNSUPPORTED) return st;
            }
        }
        if (st != SDRGPU_OK && want_os()) {
            ran = SDRGPU_FIR_OVERLAP_SAVE;
            if (!os_state && os_status == SDRGPU_OK)
                os_state = fir_os_prepare(device, csk, tk, taps_host.data(), K, D, stream.cur,
                                          &os_status);
            if (os_state) st = fir_os_launch(p, os_state, stream.cur);
            kern = SDRGPU_FIR_KERNEL_OVERLAP_SAVE;
            if (st != SDRGPU_OK && algo == SDRGPU_FIR_OVERLAP_SAVE) return st;
        }
        if (st != SDRGPU_OK) {
            ran = SDRGPU_FIR_DIRECT;
            st = fir_direct_launch(p, stream.cur);
            kern = SDRGPU_FIR_KERNEL_DIRECT;
        }
        if (st) return st;
        last_algo = ran;
        last_kernel = kern | conv;
        if (K > 1) cur ^= 1;
        seen += n_in;
        return SDRGPU_OK;
    }

    int process_host(const void* in, size_t ld_in, size_t n_in, void* out, size_t ld_out,
                     size_t out_cap, size_t* n_out_ret) {
        const size_t n_out = out_len(n_in);
        if (n_out_ret) *n_out_ret = n_out;
        if (n_out > out_cap) return SDRGPU_ERR_OUTPUT_CAP;
        if (n_in == 0) return SDRGPU_OK;
        if (!in || (n_out && !out)) return SDRGPU_ERR_INVALID;
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_ERR_DEVICE;
        const size_t ib = in_bytes(), ob = out_bytes();
        int st;
        // Stage densely (leading dimension = n_in / n_out on the device).
        if ((st = stage_in.ensure(nch * n_in * ib))) return st;
        if ((st = stage_out.ensure(nch * (n_out ? n_out : 1) * ob))) return st;
        SDRGPU_HIP_TRY(hipMemcpy2DAsync(stage_in.ptr, n_in * ib, in, ld_in * ib, n_in * ib, nch,
                                        hipMemcpyHostToDevice, stream.cur));
        size_t got = 0;
        if ((st = run_dev(stage_in.ptr, n_in, n_in, stage_out.ptr, n_out, &got))) return st;
        if (n_out)
            SDRGPU_HIP_TRY(hipMemcpy2DAsync(out, ld_out * ob, stage_out.ptr, n_out * ob,
                                            n_out * ob, nch, hipMemcpyDeviceToHost, stream.cur));
        SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
        return SDRGPU_OK;
    }

    // Host pointers, asynchronous: H2D + FIR + D2H enqueued on the handle's stream, no
    // wait.  With pinned buffers (sdrgpu_host_alloc) the copies are DMA straight from/to
    // the caller's memory, so a caller that double-buffers fills block i+1 while block i is
    // in flight -- the Block adapter's producer/consumer split (block.rs:105-207) with the
    // GPU as the consumer.  Calls on one handle are stream-ordered, so the staging buffers
    // are reused safely; `in` must stay untouched and `out` unread until *_sync.
    int process_host_async(const void* in, size_t n_in, void* out, size_t out_cap,
                           size_t* n_out_ret) {
        const size_t n_out = out_len(n_in);
        if (n_out_ret) *n_out_ret = n_out;
        if (n_out > out_cap) return SDRGPU_ERR_OUTPUT_CAP;
        if (n_in == 0) return SDRGPU_OK;
        if (!in || (n_out && !out)) return SDRGPU_ERR_INVALID;
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_ERR_DEVICE;
        const size_t ib = in_bytes(), ob = out_bytes();
        int st;
        if (!d2h) {
            SDRGPU_HIP_TRY(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
            for (int i = 0; i < 2; ++i) {
                SDRGPU_HIP_TRY(hipEventCreateWithFlags(&ev_k[i], hipEventDisableTiming));
                SDRGPU_HIP_TRY(hipEventCreateWithFlags(&ev_o[i], hipEventDisableTiming));
            }
        }
        const int slot = aslot;
        aslot ^= 1;
        DevBuf& so = stage_aout[slot];
        if (stage_in.cap < nch * n_in * ib || so.cap < nch * (n_out ? n_out : 1) * ob)
            if ((st = sync_all())) return st;  // growing frees buffers that may be in flight
        if ((st = stage_in.ensure(nch * n_in * ib))) return st;
        if ((st = so.ensure(nch * (n_out ? n_out : 1) * ob))) return st;
        SDRGPU_HIP_TRY(hipMemcpyAsync(stage_in.ptr, in, nch * n_in * ib, hipMemcpyHostToDevice,
                                      stream.cur));
        // the previous download from this slot must finish before the FIR overwrites it
        if (ev_o_live[slot]) SDRGPU_HIP_TRY(hipStreamWaitEvent(stream.cur, ev_o[slot], 0));
        size_t got = 0;
        if ((st = run_dev(stage_in.ptr, n_in, n_in, so.ptr, n_out, &got))) return st;
        if (n_out) {
            SDRGPU_HIP_TRY(hipEventRecord(ev_k[slot], stream.cur));
            SDRGPU_HIP_TRY(hipStreamWaitEvent(d2h, ev_k[slot], 0));
            SDRGPU_HIP_TRY(hipMemcpyAsync(out, so.ptr, nch * n_out * ob, hipMemcpyDeviceToHost,
                                          d2h));
            SDRGPU_HIP_TRY(hipEventRecord(ev_o[slot], d2h));
            ev_o_live[slot] = true;
        }
        return SDRGPU_OK;
    }

    int clone_into(FirCore* dst) const {
        int st = dst->init(device, sk, tk, taps_host.data(), (size_t)K, (uint32_t)D, nch);
        if (st) return st;
        DeviceGuard g(device);
        dst->algo = algo;
        dst->seen = seen;
        dst->cur = 0;
        if (K > 1) {
            SDRGPU_HIP_TRY(hipMemcpyAsync(dst->d_hist[0], d_hist[cur], hist_bytes(),
                                          hipMemcpyDeviceToDevice, stream.cur));
            SDRGPU_HIP_TRY(hipStreamSynchronize(stream.cur));
        }
        return SDRGPU_OK;
    }
};

struct sdrgpu_fir {
    FirCore core;
};
struct sdrgpu_firbank {
    FirCore core;
};

extern "C" {

// ------------------------------- single stream -------------------------------------
int sdrgpu_fir_create(int device, int sample_kind, int tap_kind, const void* taps,
                      size_t ntaps, uint32_t decim, sdrgpu_fir** out) {
    if (!out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    auto* h = new (std::nothrow) sdrgpu_fir();
    if (!h) return SDRGPU_ERR_NOMEM;
    int st = h->core.init(device, sample_kind, tap_kind, taps, ntaps, decim, 1);
    if (st) {
        h->core.free_all();
        delete h;
        return st;
    }
    *out = h;
    return SDRGPU_OK;
}

int sdrgpu_fir_set_algorithm(sdrgpu_fir* h, int algo) {
    if (!h || algo < SDRGPU_FIR_AUTO || algo > SDRGPU_FIR_MATRIX) return SDRGPU_ERR_INVALID;
    if (algo == SDRGPU_FIR_OVERLAP_SAVE &&
        !fir_os_supported(h->core.csk, h->core.tk, h->core.K, h->core.D))
        return SDRGPU_ERR_UNSUPPORTED;
    if (algo == SDRGPU_FIR_MATRIX &&
        !fir_mx_supported(h->core.csk, h->core.tk, h->core.K, h->core.D))
        return SDRGPU_ERR_UNSUPPORTED;
    h->core.algo = algo;
    return SDRGPU_OK;
}

int sdrgpu_fir_set_stream(sdrgpu_fir* h, void* s) {
    if (!h) return SDRGPU_ERR_INVALID;
    h->core.stream.set(s);
    return SDRGPU_OK;
}

int sdrgpu_fir_get_stream(const sdrgpu_fir* h, void** s) {
    if (!h || !s) return SDRGPU_ERR_INVALID;
    *s = h->core.stream.cur;
    return SDRGPU_OK;
}

int sdrgpu_fir_output_len(const sdrgpu_fir* h, size_t n_in, size_t* n_out) {
    if (!h || !n_out) return SDRGPU_ERR_INVALID;
    *n_out = h->core.out_len(n_in);
    return SDRGPU_OK;
}

int sdrgpu_fir_process(sdrgpu_fir* h, const void* in, size_t n_in, void* out, size_t out_cap,
                       size_t* n_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    return h->core.process_host(in, n_in, n_in, out, out_cap, out_cap, n_out);
}

int sdrgpu_fir_process_async(sdrgpu_fir* h, const void* in, size_t n_in, void* out,
                             size_t out_cap, size_t* n_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    return h->core.process_host_async(in, n_in, out, out_cap, n_out);
}

int sdrgpu_fir_process_dev(sdrgpu_fir* h, const void* d_in, size_t n_in, void* d_out,
                           size_t out_cap, size_t* n_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    const size_t need = h->core.out_len(n_in);
    if (n_out) *n_out = need;
    if (need > out_cap) return SDRGPU_ERR_OUTPUT_CAP;
    DeviceGuard g(h->core.device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    return h->core.run_dev(d_in, n_in, n_in, d_out, out_cap, n_out);
}

int sdrgpu_fir_sync(sdrgpu_fir* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    return h->core.sync_all();
}

int sdrgpu_fir_last_algorithm(const sdrgpu_fir* h, int* algo) {
    if (!h || !algo) return SDRGPU_ERR_INVALID;
    *algo = h->core.last_algo;
    return SDRGPU_OK;
}

int sdrgpu_fir_last_kernel(const sdrgpu_fir* h, int* kernel) {
    if (!h || !kernel) return SDRGPU_ERR_INVALID;
    *kernel = h->core.last_kernel;
    return SDRGPU_OK;
}

int sdrgpu_fir_reset(sdrgpu_fir* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    return h->core.reset_state();
}

int sdrgpu_fir_clone(const sdrgpu_fir* h, sdrgpu_fir** out) {
    if (!h || !out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    auto* c = new (std::nothrow) sdrgpu_fir();
    if (!c) return SDRGPU_ERR_NOMEM;
    int st = h->core.clone_into(&c->core);
    if (st) {
        c->core.free_all();
        delete c;
        return st;
    }
    *out = c;
    return SDRGPU_OK;
}

void sdrgpu_fir_destroy(sdrgpu_fir* h) {
    if (!h) return;
    h->core.free_all();
    delete h;
}

// ------------------------------- FIR bank ------------------------------------------
int sdrgpu_firbank_create(int device, int sample_kind, int tap_kind, const void* taps,
                          size_t ntaps, uint32_t decim, size_t nch, sdrgpu_firbank** out) {
    if (!out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    auto* h = new (std::nothrow) sdrgpu_firbank();
    if (!h) return SDRGPU_ERR_NOMEM;
    int st = h->core.init(device, sample_kind, tap_kind, taps, ntaps, decim, nch);
    if (st) {
        h->core.free_all();
        delete h;
        return st;
    }
    *out = h;
    return SDRGPU_OK;
}

int sdrgpu_firbank_set_algorithm(sdrgpu_firbank* h, int algo) {
    if (!h || algo < SDRGPU_FIR_AUTO || algo > SDRGPU_FIR_MATRIX) return SDRGPU_ERR_INVALID;
    if (algo == SDRGPU_FIR_OVERLAP_SAVE &&
        !fir_os_supported(h->core.csk, h->core.tk, h->core.K, h->core.D))
        return SDRGPU_ERR_UNSUPPORTED;
    if (algo == SDRGPU_FIR_MATRIX &&
        !fir_mx_supported(h->core.csk, h->core.tk, h->core.K, h->core.D))
        return SDRGPU_ERR_UNSUPPORTED;
    h->core.algo = algo;
    return SDRGPU_OK;
}

int sdrgpu_firbank_set_stream(sdrgpu_firbank* h, void* s) {
    if (!h) return SDRGPU_ERR_INVALID;
    h->core.stream.set(s);
    return SDRGPU_OK;
}

int sdrgpu_firbank_get_stream(const sdrgpu_firbank* h, void** s) {
    if (!h || !s) return SDRGPU_ERR_INVALID;
    *s = h->core.stream.cur;
    return SDRGPU_OK;
}

int sdrgpu_firbank_output_len(const sdrgpu_firbank* h, size_t n_in, size_t* n_out) {
    if (!h || !n_out) return SDRGPU_ERR_INVALID;
    *n_out = h->core.out_len(n_in);
    return SDRGPU_OK;
}

int sdrgpu_firbank_process(sdrgpu_firbank* h, const void* in, size_t ld_in, size_t n_in,
                           void* out, size_t ld_out, size_t* n_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    const size_t need = h->core.out_len(n_in);
    if (ld_in < n_in || (need && ld_out < need)) return SDRGPU_ERR_INVALID;
    return h->core.process_host(in, ld_in, n_in, out, ld_out, ld_out, n_out);
}

int sdrgpu_firbank_process_dev(sdrgpu_firbank* h, const void* d_in, size_t ld_in, size_t n_in,
                               void* d_out, size_t ld_out, size_t* n_out) {
    if (!h) return SDRGPU_ERR_INVALID;
    const size_t need = h->core.out_len(n_in);
    if (n_out) *n_out = need;
    if (ld_in < n_in || (need && ld_out < need)) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->core.device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    return h->core.run_dev(d_in, ld_in, n_in, d_out, ld_out, n_out);
}

int sdrgpu_firbank_sync(sdrgpu_firbank* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->core.device);
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->core.stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_firbank_last_algorithm(const sdrgpu_firbank* h, int* algo) {
    if (!h || !algo) return SDRGPU_ERR_INVALID;
    *algo = h->core.last_algo;
    return SDRGPU_OK;
}

int sdrgpu_firbank_last_kernel(const sdrgpu_firbank* h, int* kernel) {
    if (!h || !kernel) return SDRGPU_ERR_INVALID;
    *kernel = h->core.last_kernel;
    return SDRGPU_OK;
}

int sdrgpu_firbank_reset(sdrgpu_firbank* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    return h->core.reset_state();
}

int sdrgpu_firbank_clone(const sdrgpu_firbank* h, sdrgpu_firbank** out) {
    if (!h || !out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    auto* c = new (std::nothrow) sdrgpu_firbank();
    if (!c) return SDRGPU_ERR_NOMEM;
    int st = h->core.clone_into(&c->core);
    if (st) {
        c->core.free_all();
        delete c;
        return st;
    }
    *out = c;
    return SDRGPU_OK;
}

void sdrgpu_firbank_destroy(sdrgpu_firbank* h) {
    if (!h) return;
    h->core.free_all();
    delete h;
}

}  // extern "C"
