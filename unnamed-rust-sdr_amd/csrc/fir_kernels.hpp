// fir_kernels.hpp -- internal launch interface of the FIR kernels (not part of the ABI).
#pragma once

#include "common.hpp"

namespace sdrgpu {

// Taps are kept on the device in polyphase-major order: taps_pm[p*tpp + i] = h[p + i*D]
// (zero beyond K), tpp = ceil(ceil(K/D) / 16) * 16.
constexpr int kTapPad = 16;

inline int taps_per_phase(int K, int D) {
    int t = (K + D - 1) / D;
    return (t + kTapPad - 1) / kTapPad * kTapPad;
}

struct FirParams {
    int sample_kind, tap_kind;
    const void* in;       // device, channel c at in + c*ld_in samples
    long ld_in;
    long n_in;            // samples this call, per channel
    const void* hist;     // device, nch x (K-1): stream samples -(K-1)..-1
    void* hist_next;      // device, written with the new history
    long i0;              // local index of the first kept output
    long n_out;           // kept outputs this call, per channel
    int K, D;
    const void* taps_pm;  // device, polyphase-major padded taps
    int tpp;
    void* out;            // device, channel c at out + c*ld_out samples
    long ld_out;
    int nch;
    int force_naive;
};

int fir_direct_launch(const FirParams& p, hipStream_t s);

// Wave-private persistent direct form (fir_direct2.hip): c64 samples, f32 taps,
// D in {1,2,4,8}, D*tpp <= 1024.  Returns SDRGPU_ERR_UNSUPPORTED otherwise.
bool fir_direct2_supported(const FirParams& p);
int fir_direct2_launch(const FirParams& p, hipStream_t s);

// Overlap-save (polyphase, LDS-resident FFT) path; returns SDRGPU_ERR_UNSUPPORTED for
// shapes it does not cover (caller falls back to direct).
struct FirOsPlan;
int fir_os_supported(int sample_kind, int tap_kind, int K, int D);

// LDS-staged direct form on a per-tile scaled two-way fp16 split, two waves per SIMD
// (fir_mxh.hip): D = 4 (K <= 257, also u8 input), D = 2 (K <= 257) and D = 1 (K <= 273).  tap_scale_exp:
// taps are multiplied by 2^tap_scale_exp before the split.  d_dummy: fir_mxh_dummy_bytes()
// of zeroed device memory (target of the clamped prefetches at a stream's end).
size_t fir_mxh_dummy_bytes();
int fir_mxh_supported(const FirParams& p);
int fir_mxh_shape_ok(int sample_kind, int tap_kind, int K, int D);  // c64: D in {1, 2, 4}; u8: D = 4
int fir_mxh_launch(const FirParams& p, const float* d_taps, int tap_scale_exp,
                   const void* d_dummy, int cus, hipStream_t s);

}  // namespace sdrgpu
