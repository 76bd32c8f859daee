// abi_common.hpp -- host-side plumbing shared by the C-ABI translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstring>
#include <utility>

#include "common.hpp"

namespace sdrgpu {
namespace detail {

// Sets the current device for the scope of one ABI call, restores it afterwards.
class DeviceGuard {
public:
    explicit DeviceGuard(int dev) {
        ok_ = hipGetDevice(&prev_) == hipSuccess && hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (ok_) (void)hipSetDevice(prev_);
    }
    bool ok() const { return ok_; }

private:
    int prev_ = 0;
    bool ok_ = false;
};

int check_device(int dev);

// Grow-only device scratch buffer.
struct DevBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return SDRGPU_OK;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
        if (bytes == 0) return SDRGPU_OK;
        if (hipMalloc(&ptr, bytes) != hipSuccess) return SDRGPU_ERR_NOMEM;
        cap = bytes;
        return SDRGPU_OK;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// Stream ownership: each handle creates its own non-blocking stream; set_stream may
// substitute an external one (not owned).
struct StreamSlot {
    hipStream_t own = nullptr;
    hipStream_t cur = nullptr;
    int create() {
        if (hipStreamCreateWithFlags(&own, hipStreamNonBlocking) != hipSuccess)
            return SDRGPU_ERR_DEVICE;
        cur = own;
        return SDRGPU_OK;
    }
    void set(void* s) { cur = s ? static_cast<hipStream_t>(s) : own; }
    void destroy() {
        if (own) (void)hipStreamDestroy(own);
        own = cur = nullptr;
    }
};

// Asynchronous host streaming (the Block adapter's producer/consumer split,
// src/signal/adapters/block.rs:105-207, with the GPU as the consumer): a block's H2D and
// kernel go on the handle's stream, its download on a second stream, so block i's D2H
// overlaps block i+1's H2D (PCIe is full duplex).  Two output slots of device staging, each
// guarded by an event: a slot is rewritten only after its previous download finished.
struct AsyncD2H {
    static constexpr int kSlots = 2, kArrays = 2;
    hipStream_t d2h = nullptr;
    hipEvent_t ev_k[kSlots] = {}, ev_o[kSlots] = {};
    bool live[kSlots] = {};
    DevBuf out[kSlots][kArrays];
    int next = 0;

    int init() {
        if (d2h) return SDRGPU_OK;
        if (hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking) != hipSuccess) return SDRGPU_ERR_DEVICE;
        for (int i = 0; i < kSlots; ++i)
            if (hipEventCreateWithFlags(&ev_k[i], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ev_o[i], hipEventDisableTiming) != hipSuccess)
                return SDRGPU_ERR_DEVICE;
        return SDRGPU_OK;
    }
    // next slot with `bytes[a]` of device staging per output array; `s` (the compute stream)
    // waits for the slot's previous download before anything later on it writes the slot
    int acquire(hipStream_t s, const size_t* bytes, int narrays, int* slot) {
        int st = init();
        if (st) return st;
        const int k = next;
        next = (next + 1) % kSlots;
        for (int a = 0; a < narrays; ++a)
            if (out[k][a].cap < bytes[a]) {
                if (hipStreamSynchronize(d2h) != hipSuccess) return SDRGPU_ERR_DEVICE;
                live[k] = false;
                if ((st = out[k][a].ensure(bytes[a]))) return st;
            }
        if (live[k] && hipStreamWaitEvent(s, ev_o[k], 0) != hipSuccess) return SDRGPU_ERR_DEVICE;
        *slot = k;
        return SDRGPU_OK;
    }
    // after the producing kernel on `s`: the download stream waits for it
    int begin_download(hipStream_t s, int slot) {
        if (hipEventRecord(ev_k[slot], s) != hipSuccess ||
            hipStreamWaitEvent(d2h, ev_k[slot], 0) != hipSuccess)
            return SDRGPU_ERR_DEVICE;
        return SDRGPU_OK;
    }
    int end_download(int slot) {
        if (hipEventRecord(ev_o[slot], d2h) != hipSuccess) return SDRGPU_ERR_DEVICE;
        live[slot] = true;
        return SDRGPU_OK;
    }
    int sync() {
        if (d2h && hipStreamSynchronize(d2h) != hipSuccess) return SDRGPU_ERR_DEVICE;
        return SDRGPU_OK;
    }
    void release() {
        if (d2h) (void)hipStreamSynchronize(d2h);
        for (int i = 0; i < kSlots; ++i) {
            for (auto& b : out[i]) b.release();
            if (ev_k[i]) (void)hipEventDestroy(ev_k[i]);
            if (ev_o[i]) (void)hipEventDestroy(ev_o[i]);
            ev_k[i] = ev_o[i] = nullptr;
            live[i] = false;
        }
        if (d2h) (void)hipStreamDestroy(d2h);
        d2h = nullptr;
    }
};

// BiquadD::design -> Biquad::new coefficients b0 b1 b2 na1 na2 (abi_pll.cpp)
int bq_design(const sdrgpu_biquad_design& d, float rate, float* c, int* ident);

inline size_t kind_bytes(int kind) { return kind == SDRGPU_C64 ? 8 : (kind == SDRGPU_CU8 ? 2 : 4); }

// Bytes spanned by rows rows of n elements (elem bytes each) with a leading dimension ld.
inline size_t rows_span(size_t rows, size_t ld, size_t n, size_t elem) {
    return rows ? ((rows - 1) * ld + n) * elem : 0;
}
// Whether the byte ranges [a, a + na) and [b, b + nb) overlap.  The time-parallel biquad and PLL
// plans read input samples after outputs were stored (warm-ups reach into the previous segment;
// the re-run and walk kernels re-read whole segments), so an in-place call takes the serial pass,
// which reads every chunk before it stores it.
inline bool bytes_overlap(const void* a, size_t na, const void* b, size_t nb) {
    const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
    return na && nb && x < y + nb && y < x + na;
}
// The FIR, FFT and STFT kernels store output tiles while other workgroups still read the input
// under them, so a device input range that overlaps the call's output range is copied to `stage`
// (on the call's stream, ahead of the kernels) and the copy is read instead: in-place calls give
// the results of out-of-place ones, at the cost of one device copy of the input.
inline int unalias_input(DevBuf& stage, const void*& in, size_t in_bytes, const void* out,
                         size_t out_bytes, hipStream_t s) {
    if (!bytes_overlap(in, in_bytes, out, out_bytes)) return SDRGPU_OK;
    const int st = stage.ensure(in_bytes);
    if (st) return st;
    if (hipMemcpyAsync(stage.ptr, in, in_bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return SDRGPU_ERR_DEVICE;
    in = stage.ptr;
    return SDRGPU_OK;
}

}  // namespace detail
}  // namespace sdrgpu
