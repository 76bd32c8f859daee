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

// BiquadD::design -> Biquad::new coefficients b0 b1 b2 na1 na2 (abi_pll.cpp)
int bq_design(const sdrgpu_biquad_design& d, float rate, float* c, int* ident);

inline size_t kind_bytes(int kind) { return kind == SDRGPU_C64 ? 8 : (kind == SDRGPU_CU8 ? 2 : 4); }

}  // namespace detail
}  // namespace sdrgpu
