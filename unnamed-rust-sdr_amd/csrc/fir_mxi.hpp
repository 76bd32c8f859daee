// fir_mxi.hpp -- launch interface of the int8-MFMA rtl_tcp u8 FIR kernel (fir_mxi.hip).
#pragma once

#include "fir_kernels.hpp"

namespace sdrgpu {

// rtl_tcp u8 input, D = 8, 4, 2 or 1, K <= 257, real taps on the int8 MFMAs: taps as three int8 digits
// of rint(h 2^(tap_scale_exp + 7)); finite taps only (the caller checks).  d_dummy: the same
// zeroed fir_mxh_dummy_bytes() buffer as fir_mxh.  16-byte aligned channel bases.
int fir_mxi_supported(const FirParams& p, int tap_scale_exp);
int fir_mxi_launch(const FirParams& p, const float* d_taps, int tap_scale_exp,
                   const void* d_dummy, int cus, hipStream_t s);

}  // namespace sdrgpu
