// fir_os.hip -- overlap-save FIR (placeholder until the LDS FFT tile kernel lands).
#include "fir_kernels.hpp"

namespace sdrgpu {

int fir_os_supported(int, int, int, int) { return 0; }

void* fir_os_prepare(int, int, int, const void*, int, int, hipStream_t, int* status) {
    if (status) *status = SDRGPU_ERR_UNSUPPORTED;
    return nullptr;
}

int fir_os_launch(const FirParams&, void*, hipStream_t) { return SDRGPU_ERR_UNSUPPORTED; }

void fir_os_release(void*) {}

}  // namespace sdrgpu
