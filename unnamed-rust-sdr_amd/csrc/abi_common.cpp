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
