// ingest.hip -- rtl_tcp u8 IQ -> Complex<f32> for the FIR shapes the fused MFMA ingest
// (fir_mxh.hip, U8) does not cover.  Replaces RtlTcpSignal::next (reference
// src/rtltcp.rs:156-164): re = (i as f32 - 128.0) / 128.0, im likewise -- exact in f32.
#include <algorithm>

#include "common.hpp"

namespace sdrgpu {

namespace {

__global__ __launch_bounds__(256) void cu8_to_c64_kernel(const unsigned short* __restrict__ in,
                                                         long ld_in, long n, long total,
                                                         float2* __restrict__ out) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long c = i / n, j = i - c * n;
        const unsigned w = in[c * ld_in + j];
        out[i] = make_float2(((float)(w & 0xffu) - 128.0f) / 128.0f,
                             ((float)(w >> 8) - 128.0f) / 128.0f);
    }
}

}  // namespace

// nch channels of n samples (channel c at in + 2*c*ld_in bytes) -> dense C64 (ld = n)
int cu8_to_c64_launch(const void* in, long ld_in, long n, long nch, void* out, hipStream_t s) {
    const long total = n * nch;
    if (total <= 0) return SDRGPU_OK;
    const long blocks = std::min<long>(ceil_div(total, 256), 8192);
    hipLaunchKernelGGL(cu8_to_c64_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       static_cast<const unsigned short*>(in), ld_in, n, total,
                       static_cast<float2*>(out));
    SDRGPU_LAUNCH_CHECK();
    return SDRGPU_OK;
}

}  // namespace sdrgpu
