// resample_kernels.hpp -- descriptors and launchers shared by abi_resample.cpp and
// resample.hip (libsamplerate converters behind src/resample.rs).
#pragma once
#include <hip/hip_runtime.h>

namespace sdrgpu {

// One sinc output frame (src_sinc.c calc_output_multi after the host's bookkeeping).
struct SincDesc {
    int dl, dr;    // window sample index (channel 0) of the first left / right tap
    int fil, fir;  // fixed-point filter index (12 fraction bits) of that tap
    int nl, nr;    // tap counts
    int inc, pad;  // fixed-point increment
    double scale;  // float_increment / index_inc
};

int src_interp_launch(bool linear, const float* in, long channels, const int* left,
                      const double* frac, long nframes, const float* last_value, float* out,
                      hipStream_t s);
int src_sinc_launch(const float* win, long channels, const SincDesc* desc, long nframes,
                    const float* coeffs, int coeff_len, float* out, hipStream_t s);

}  // namespace sdrgpu
