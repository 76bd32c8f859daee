// abi_common.cpp -- status strings, device queries (sdrgpu.h).
#include "abi_common.hpp"

namespace sdrgpu {
namespace detail {

static thread_local hipError_t g_last_hip = hipSuccess;

void set_last_hip_error(hipError_t e) { g_last_hip = e; }

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SDRGPU_ERR_NODEVICE;
    if (dev < 0 || dev >= n) return SDRGPU_ERR_NODEVICE;
    return SDRGPU_OK;
}

}  // namespace detail
}  // namespace sdrgpu

extern "C" {

// Mirrors resample::Error's Display strings in spirit (src/resample.rs:209-269).
const char* sdrgpu_strerror(int code) {
    switch (code) {
    case SDRGPU_OK: return "no error";
    case SDRGPU_ERR_INVALID: return "invalid argument";
    case SDRGPU_ERR_NOMEM: return "out of memory";
    case SDRGPU_ERR_DEVICE: return "HIP runtime error";
    case SDRGPU_ERR_NODEVICE: return "no such GPU device";
    case SDRGPU_ERR_UNSUPPORTED: return "unsupported configuration";
    case SDRGPU_ERR_OUTPUT_CAP: return "output buffer too small";
    case SDRGPU_ERR_LAUNCH: return "kernel launch failed";
    default: return "unknown error";
    }
}

int sdrgpu_abi_version(void) { return SDRGPU_ABI_VERSION; }

int sdrgpu_device_count(int* count) {
    if (!count) return SDRGPU_ERR_INVALID;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return SDRGPU_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------
// Device memory / events (sdrgpu.h "device memory, streams and timing").
extern "C" {

int sdrgpu_dev_alloc(int device, size_t bytes, void** dptr) {
    using namespace sdrgpu::detail;
    if (!dptr) return SDRGPU_ERR_INVALID;
    *dptr = nullptr;
    int st = check_device(device);
    if (st) return st;
    DeviceGuard g(device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    SDRGPU_HIP_TRY(hipMalloc(dptr, bytes ? bytes : 1));
    return SDRGPU_OK;
}

int sdrgpu_host_alloc(int device, size_t bytes, void** hptr) {
    using namespace sdrgpu::detail;
    if (!hptr) return SDRGPU_ERR_INVALID;
    *hptr = nullptr;
    int st = check_device(device);
    if (st) return st;
    DeviceGuard g(device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    if (hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
        return SDRGPU_ERR_NOMEM;
    return SDRGPU_OK;
}

int sdrgpu_host_free(void* hptr) {
    if (!hptr) return SDRGPU_OK;
    SDRGPU_HIP_TRY(hipHostFree(hptr));
    return SDRGPU_OK;
}

int sdrgpu_dev_free(int device, void* dptr) {
    using namespace sdrgpu::detail;
    if (!dptr) return SDRGPU_OK;
    DeviceGuard g(device);
    SDRGPU_HIP_TRY(hipFree(dptr));
    return SDRGPU_OK;
}

int sdrgpu_dev_copy(int device, void* dst, const void* src, size_t bytes, int kind) {
    using namespace sdrgpu::detail;
    if ((!dst || !src) && bytes) return SDRGPU_ERR_INVALID;
    hipMemcpyKind k;
    switch (kind) {
    case SDRGPU_H2D: k = hipMemcpyHostToDevice; break;
    case SDRGPU_D2H: k = hipMemcpyDeviceToHost; break;
    case SDRGPU_D2D: k = hipMemcpyDeviceToDevice; break;
    default: return SDRGPU_ERR_INVALID;
    }
    if (!bytes) return SDRGPU_OK;
    DeviceGuard g(device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    SDRGPU_HIP_TRY(hipMemcpy(dst, src, bytes, k));
    return SDRGPU_OK;
}

int sdrgpu_dev_memset(int device, void* dptr, int value, size_t bytes) {
    using namespace sdrgpu::detail;
    if (!dptr && bytes) return SDRGPU_ERR_INVALID;
    if (!bytes) return SDRGPU_OK;
    DeviceGuard g(device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    SDRGPU_HIP_TRY(hipMemset(dptr, value, bytes));
    return SDRGPU_OK;
}

int sdrgpu_dev_synchronize(int device) {
    using namespace sdrgpu::detail;
    int st = check_device(device);
    if (st) return st;
    DeviceGuard g(device);
    SDRGPU_HIP_TRY(hipDeviceSynchronize());
    return SDRGPU_OK;
}

int sdrgpu_event_create(int device, void** event) {
    using namespace sdrgpu::detail;
    if (!event) return SDRGPU_ERR_INVALID;
    *event = nullptr;
    int st = check_device(device);
    if (st) return st;
    DeviceGuard g(device);
    hipEvent_t e;
    SDRGPU_HIP_TRY(hipEventCreate(&e));
    *event = e;
    return SDRGPU_OK;
}

int sdrgpu_event_record(void* event, void* stream) {
    if (!event) return SDRGPU_ERR_INVALID;
    SDRGPU_HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(event), static_cast<hipStream_t>(stream)));
    return SDRGPU_OK;
}

int sdrgpu_event_synchronize(void* event) {
    if (!event) return SDRGPU_ERR_INVALID;
    SDRGPU_HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    return SDRGPU_OK;
}

int sdrgpu_event_elapsed_ms(void* start, void* end, float* ms) {
    if (!start || !end || !ms) return SDRGPU_ERR_INVALID;
    SDRGPU_HIP_TRY(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start),
                                       static_cast<hipEvent_t>(end)));
    return SDRGPU_OK;
}

int sdrgpu_event_destroy(void* event) {
    if (!event) return SDRGPU_OK;
    SDRGPU_HIP_TRY(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return SDRGPU_OK;
}

}  // extern "C"
