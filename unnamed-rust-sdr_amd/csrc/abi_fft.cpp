// abi_fft.cpp -- C ABI of the FFT (fft::fft / fft::rfft, reference src/fft.rs:3-37) and the
// streaming STFT (Window + Decimate + fft, src/signal/adapters/mod.rs:13-41,270-303 as
// composed in examples/live.rs:29-39).
#include <vector>

#include "abi_common.hpp"
#include "fft_kernels.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

struct sdrgpu_fft {
    int device = 0;
    int n = 0;
    int out_db = 0;  // SDRGPU_FFT_OUT_DB: f32 dB magnitudes instead of C64 values
    void* plan = nullptr;
    StreamSlot stream;
    DevBuf stage_in, stage_out, scratch, alias;  // alias: copy of an input the output overlaps
    AsyncD2H async;
    size_t out_elem() const { return out_db ? sizeof(float) : sizeof(float2); }

    int ensure_scratch() {
        const size_t b = fft_scratch_bytes(plan);
        if (!b) return SDRGPU_OK;
        return scratch.ensure(b);
    }
    void free_all() {
        DeviceGuard g(device);
        stage_in.release();
        stage_out.release();
        scratch.release();
        alias.release();
        async.release();
        if (plan) fft_plan_destroy(plan);
        plan = nullptr;
        stream.destroy();
    }
    int run(const FftFrames& fr, float2* out, int store_mode) {
        int st = ensure_scratch();
        if (st) return st;
        if (out_db) store_mode += 3;  // collated / rfft as dB magnitudes
        return fft_launch(plan, fr, out, store_mode, static_cast<float2*>(scratch.ptr),
                          fft_scratch_frames(plan), stream.cur);
    }
};

static int fft_init(sdrgpu_fft* h, int device, size_t n) {
    int st = check_device(device);
    if (st) return st;
    h->device = device;
    h->n = (int)n;
    DeviceGuard g(device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    if ((st = h->stream.create())) return st;
    h->plan = fft_plan_create((int)n, &st);
    return st;
}

struct sdrgpu_stft {
    sdrgpu_fft fft;
    long hop = 1;
    long H = 0;  // n - 1 history samples
    int in_kind = SDRGPU_C64;  // or SDRGPU_CU8 (rtl_tcp bytes, converted in the frame load)
    float2* d_hist[2] = {nullptr, nullptr};
    int cur = 0;
    unsigned long long seen = 0;

    size_t frames_for(size_t n_in) const {
        const unsigned long long h = (unsigned long long)hop;
        return (size_t)((seen + n_in) / h - seen / h);
    }
    long first_end() const { return hop - (long)(seen % (unsigned long long)hop); }
};

extern "C" {

int sdrgpu_fft_plan(int device, size_t n, sdrgpu_fft** out) {
    if (!out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    if (n == 0) return SDRGPU_ERR_INVALID;
    if (n > (1u << 24)) return SDRGPU_ERR_UNSUPPORTED;
    auto* h = new (std::nothrow) sdrgpu_fft();
    if (!h) return SDRGPU_ERR_NOMEM;
    int st = fft_init(h, device, n);
    if (st) {
        h->free_all();
        delete h;
        return st;
    }
    *out = h;
    return SDRGPU_OK;
}

int sdrgpu_fft_set_stream(sdrgpu_fft* h, void* s) {
    if (!h) return SDRGPU_ERR_INVALID;
    h->stream.set(s);
    return SDRGPU_OK;
}

int sdrgpu_fft_get_stream(const sdrgpu_fft* h, void** s) {
    if (!h || !s) return SDRGPU_ERR_INVALID;
    *s = h->stream.cur;
    return SDRGPU_OK;
}

int sdrgpu_fft_exec_dev(sdrgpu_fft* h, const void* d_in, void* d_out, size_t count) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (count == 0) return SDRGPU_OK;
    if (!d_in || !d_out) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    int st = unalias_input(h->alias, d_in, count * (size_t)h->n * sizeof(float2), d_out,
                           count * (size_t)h->n * h->out_elem(), h->stream.cur);
    if (st) return st;
    FftFrames fr{};
    fr.mode = 0;
    fr.in = static_cast<const float2*>(d_in);
    fr.nframes = (long)count;
    return h->run(fr, static_cast<float2*>(d_out), 0);
}

int sdrgpu_fft_exec(sdrgpu_fft* h, const void* in, void* out, size_t count) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (count == 0) return SDRGPU_OK;
    if (!in || !out) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const size_t bytes = count * (size_t)h->n * sizeof(float2);
    const size_t obytes = count * (size_t)h->n * h->out_elem();
    int st;
    if ((st = h->stage_in.ensure(bytes)) || (st = h->stage_out.ensure(obytes))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(h->stage_in.ptr, in, bytes, hipMemcpyHostToDevice, h->stream.cur));
    if ((st = sdrgpu_fft_exec_dev(h, h->stage_in.ptr, h->stage_out.ptr, count))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(out, h->stage_out.ptr, obytes, hipMemcpyDeviceToHost, h->stream.cur));
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_rfft_exec_dev(sdrgpu_fft* h, const float* d_in, void* d_out, size_t count) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (count == 0) return SDRGPU_OK;
    if (!d_in || !d_out) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const void* in = d_in;
    int st = unalias_input(h->alias, in, count * (size_t)h->n * sizeof(float), d_out,
                           count * (size_t)(h->n - h->n / 2) * h->out_elem(), h->stream.cur);
    if (st) return st;
    FftFrames fr{};
    fr.mode = 2;
    fr.in_real = static_cast<const float*>(in);
    fr.nframes = (long)count;
    return h->run(fr, static_cast<float2*>(d_out), 1);
}

int sdrgpu_rfft_exec(sdrgpu_fft* h, const float* in, void* out, size_t count) {
    if (!h) return SDRGPU_ERR_INVALID;
    if (count == 0) return SDRGPU_OK;
    if (!in || !out) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const size_t in_bytes = count * (size_t)h->n * sizeof(float);
    const size_t out_bytes = count * (size_t)(h->n - h->n / 2) * h->out_elem();
    int st;
    if ((st = h->stage_in.ensure(in_bytes)) || (st = h->stage_out.ensure(out_bytes))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(h->stage_in.ptr, in, in_bytes, hipMemcpyHostToDevice, h->stream.cur));
    if ((st = sdrgpu_rfft_exec_dev(h, static_cast<const float*>(h->stage_in.ptr), h->stage_out.ptr, count)))
        return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(out, h->stage_out.ptr, out_bytes, hipMemcpyDeviceToHost, h->stream.cur));
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_fft_set_output(sdrgpu_fft* h, int mode) {
    if (!h || (mode != SDRGPU_FFT_OUT_COMPLEX && mode != SDRGPU_FFT_OUT_DB)) return SDRGPU_ERR_INVALID;
    h->out_db = mode == SDRGPU_FFT_OUT_DB;
    return SDRGPU_OK;
}

int sdrgpu_fft_sync(sdrgpu_fft* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->device);
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->stream.cur));
    return h->async.sync();
}

void sdrgpu_fft_destroy(sdrgpu_fft* h) {
    if (!h) return;
    h->free_all();
    delete h;
}

// fft.rs:18,24: freq = (i - n/2) as f32 * (rate / n as f32)
int sdrgpu_fft_freqs(size_t n, float rate, float* freqs) {
    if (!freqs || n == 0) return SDRGPU_ERR_INVALID;
    const float fstep = rate / (float)n;
    const long start = -(long)(n / 2);
    for (size_t i = 0; i < n; ++i) freqs[i] = (float)(start + (long)i) * fstep;
    return SDRGPU_OK;
}

// ----------------------------------- STFT ------------------------------------------
int sdrgpu_stft_create(int device, size_t n, size_t hop, sdrgpu_stft** out) {
    if (!out) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    if (n == 0 || hop == 0) return SDRGPU_ERR_INVALID;
    if (n > (1u << 24)) return SDRGPU_ERR_UNSUPPORTED;
    auto* h = new (std::nothrow) sdrgpu_stft();
    if (!h) return SDRGPU_ERR_NOMEM;
    int st = fft_init(&h->fft, device, n);
    if (!st) {
        h->hop = (long)hop;
        h->H = (long)n - 1;
        DeviceGuard g(device);
        if (hipMalloc(&h->d_hist[0], h->H * sizeof(float2)) != hipSuccess ||
            hipMalloc(&h->d_hist[1], h->H * sizeof(float2)) != hipSuccess)
            st = SDRGPU_ERR_NOMEM;
        else
            st = sdrgpu_stft_reset(h);
    }
    if (st) {
        sdrgpu_stft_destroy(h);
        return st;
    }
    *out = h;
    return SDRGPU_OK;
}

int sdrgpu_stft_set_stream(sdrgpu_stft* h, void* s) {
    if (!h) return SDRGPU_ERR_INVALID;
    h->fft.stream.set(s);
    return SDRGPU_OK;
}

int sdrgpu_stft_get_stream(const sdrgpu_stft* h, void** s) {
    if (!h || !s) return SDRGPU_ERR_INVALID;
    *s = h->fft.stream.cur;
    return SDRGPU_OK;
}

int sdrgpu_stft_output_len(const sdrgpu_stft* h, size_t n_in, size_t* n_frames) {
    if (!h || !n_frames) return SDRGPU_ERR_INVALID;
    *n_frames = h->frames_for(n_in);
    return SDRGPU_OK;
}

int sdrgpu_stft_process_dev(sdrgpu_stft* h, const void* d_in, size_t n_in, void* d_out,
                            size_t out_cap_frames, size_t* n_frames) {
    if (!h) return SDRGPU_ERR_INVALID;
    const size_t nf = h->frames_for(n_in);
    if (n_frames) *n_frames = nf;
    if (nf > out_cap_frames) return SDRGPU_ERR_OUTPUT_CAP;
    if (n_in == 0) return SDRGPU_OK;
    if (!d_in || (nf && !d_out)) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->fft.device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    // the frames are stored before the carry kernel re-reads the input's tail
    int st = unalias_input(h->fft.alias, d_in, n_in * kind_bytes(h->in_kind), d_out,
                           nf * (size_t)h->fft.n * h->fft.out_elem(), h->fft.stream.cur);
    if (st) return st;
    FftFrames fr{};
    const bool u8 = h->in_kind == SDRGPU_CU8;
    fr.mode = u8 ? 3 : 1;
    fr.in = static_cast<const float2*>(d_in);
    fr.in_u8 = static_cast<const unsigned short*>(d_in);
    fr.n_in = (long)n_in;
    fr.hist = h->d_hist[h->cur];
    fr.H = h->H;
    fr.first_end = h->first_end();
    fr.hop = h->hop;
    fr.nframes = (long)nf;
    st = h->fft.run(fr, static_cast<float2*>(d_out), 0);
    if (st) return st;
    st = u8 ? stft_carry_u8_launch(fr.in_u8, fr.n_in, h->d_hist[h->cur], h->d_hist[h->cur ^ 1],
                                   h->H, h->fft.stream.cur)
            : stft_carry_launch(fr.in, fr.n_in, h->d_hist[h->cur], h->d_hist[h->cur ^ 1], h->H,
                                h->fft.stream.cur);
    if (st) return st;
    h->cur ^= 1;
    h->seen += n_in;
    return SDRGPU_OK;
}

int sdrgpu_stft_process(sdrgpu_stft* h, const void* in, size_t n_in, void* out,
                        size_t out_cap_frames, size_t* n_frames) {
    if (!h) return SDRGPU_ERR_INVALID;
    const size_t nf = h->frames_for(n_in);
    if (n_frames) *n_frames = nf;
    if (nf > out_cap_frames) return SDRGPU_ERR_OUTPUT_CAP;
    if (n_in == 0) return SDRGPU_OK;
    if (!in || (nf && !out)) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->fft.device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    const size_t ib = n_in * kind_bytes(h->in_kind), ob = nf * (size_t)h->fft.n * h->fft.out_elem();
    int st;
    if ((st = h->fft.stage_in.ensure(ib)) || (st = h->fft.stage_out.ensure(ob ? ob : 8))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(h->fft.stage_in.ptr, in, ib, hipMemcpyHostToDevice, h->fft.stream.cur));
    size_t got = 0;
    if ((st = sdrgpu_stft_process_dev(h, h->fft.stage_in.ptr, n_in, h->fft.stage_out.ptr, nf, &got)))
        return st;
    if (ob)
        SDRGPU_HIP_TRY(hipMemcpyAsync(out, h->fft.stage_out.ptr, ob, hipMemcpyDeviceToHost, h->fft.stream.cur));
    SDRGPU_HIP_TRY(hipStreamSynchronize(h->fft.stream.cur));
    return SDRGPU_OK;
}

int sdrgpu_stft_process_async(sdrgpu_stft* h, const void* in, size_t n_in, void* out,
                              size_t out_cap_frames, size_t* n_frames) {
    if (!h) return SDRGPU_ERR_INVALID;
    const size_t nf = h->frames_for(n_in);
    if (n_frames) *n_frames = nf;
    if (nf > out_cap_frames) return SDRGPU_ERR_OUTPUT_CAP;
    if (n_in == 0) return SDRGPU_OK;
    if (!in || (nf && !out)) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->fft.device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    sdrgpu_fft& f = h->fft;
    const size_t ib = n_in * kind_bytes(h->in_kind), ob = nf * (size_t)f.n * f.out_elem();
    int st, slot = 0;
    if (f.stage_in.cap < ib) {  // growing frees a buffer an earlier block may still read
        SDRGPU_HIP_TRY(hipStreamSynchronize(f.stream.cur));
        if ((st = f.stage_in.ensure(ib))) return st;
    }
    const size_t obytes[1] = {ob ? ob : 8};
    if ((st = f.async.acquire(f.stream.cur, obytes, 1, &slot))) return st;
    SDRGPU_HIP_TRY(hipMemcpyAsync(f.stage_in.ptr, in, ib, hipMemcpyHostToDevice, f.stream.cur));
    size_t got = 0;
    if ((st = sdrgpu_stft_process_dev(h, f.stage_in.ptr, n_in, f.async.out[slot][0].ptr, nf, &got)))
        return st;
    if (ob) {
        if ((st = f.async.begin_download(f.stream.cur, slot))) return st;
        SDRGPU_HIP_TRY(hipMemcpyAsync(out, f.async.out[slot][0].ptr, ob, hipMemcpyDeviceToHost,
                                      f.async.d2h));
        if ((st = f.async.end_download(slot))) return st;
    }
    return SDRGPU_OK;
}

int sdrgpu_stft_set_input_kind(sdrgpu_stft* h, int sample_kind) {
    if (!h || (sample_kind != SDRGPU_C64 && sample_kind != SDRGPU_CU8)) return SDRGPU_ERR_INVALID;
    h->in_kind = sample_kind;
    return SDRGPU_OK;
}

int sdrgpu_stft_set_output(sdrgpu_stft* h, int mode) {
    if (!h) return SDRGPU_ERR_INVALID;
    return sdrgpu_fft_set_output(&h->fft, mode);
}

int sdrgpu_stft_sync(sdrgpu_stft* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    int st = sdrgpu_fft_sync(&h->fft);
    if (st) return st;
    DeviceGuard g(h->fft.device);
    return h->fft.async.sync();
}

int sdrgpu_stft_reset(sdrgpu_stft* h) {
    if (!h) return SDRGPU_ERR_INVALID;
    DeviceGuard g(h->fft.device);
    h->seen = 0;
    h->cur = 0;
    if (h->H > 0) {
        SDRGPU_HIP_TRY(hipMemsetAsync(h->d_hist[0], 0, h->H * sizeof(float2), h->fft.stream.cur));
        SDRGPU_HIP_TRY(hipStreamSynchronize(h->fft.stream.cur));
    }
    return SDRGPU_OK;
}

void sdrgpu_stft_destroy(sdrgpu_stft* h) {
    if (!h) return;
    {
        DeviceGuard g(h->fft.device);
        for (auto& p : h->d_hist)
            if (p) (void)hipFree(p);
    }
    h->fft.free_all();
    delete h;
}

}  // extern "C"
