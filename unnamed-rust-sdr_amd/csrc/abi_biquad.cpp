// abi_biquad.cpp -- C ABI of the batched biquad: BiquadD::design + Biquad::new/apply
// (reference src/filter/biquad.rs:25-56, 73-155), Identity (src/filter/simple.rs:3-19), driven
// as Signal::filter (src/signal/mod.rs:42-48) on nch independent channels.  State (x1, x2,
// y1, y2 per channel) carries across calls; clone copies it (#[derive(Clone)], biquad.rs:4).
#include <cstring>

#include "abi_common.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

namespace sdrgpu {
struct BiquadState {
    float x1r, x1i, x2r, x2i, y1r, y1i, y2r, y2i;
};
int biquad_launch(bool cplx, long nch, const float* c, int ident, const void* in, long ld_in,
                  long n, void* out, long ld_out, BiquadState* state, hipStream_t s);
}  // namespace sdrgpu

struct sdrgpu_biquad {
    int device = 0, sk = SDRGPU_F32, ident = 0;
    size_t nch = 1;
    float c[5] = {1.f, 0.f, 0.f, 0.f, 0.f};
    BiquadState* d_state = nullptr;
    StreamSlot stream;
    DevBuf stage_in, stage_out;

    size_t sbytes() const { return kind_bytes(sk); }
    void free_all() {
        DeviceGuard g(device);
        if (d_state) (void)hipFree(d_state);
        d_state = nullptr;
        stage_in.release();
        stage_out.release();
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
        return reset();
    }
    int run_dev(const void* in, size_t ld_in, size_t n, void* out, size_t ld_out) {
        if (n == 0) return SDRGPU_OK;
        if (!in || !out || ld_in < n || ld_out < n) return SDRGPU_ERR_INVALID;
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
