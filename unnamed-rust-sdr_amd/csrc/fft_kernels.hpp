// fft_kernels.hpp -- internal launch interface of the FFT / STFT kernels.
#pragma once

#include "common.hpp"

namespace sdrgpu {

// Frame source description (see fft.hip FrameSrc).
struct FftFrames {
    int mode;              // 0 contiguous c64 frames, 1 STFT frames from a stream, 2 real frames,
                           // 3 STFT frames from a u8 I/Q stream
    const float2* in;
    const float* in_real;
    const unsigned short* in_u8;
    long n_in;             // stream samples in this call (mode 1)
    const float2* hist;    // H previous stream samples (mode 1)
    long H;
    long first_end;        // local stream index (exclusive) where frame 0 ends (mode 1)
    long hop;
    long nframes;
};

void* fft_plan_create(int M, int* status);
void fft_plan_destroy(void* plan);
int fft_plan_size(void* plan);
size_t fft_scratch_frames(void* plan);  // frames per batch; 0 if no scratch is needed
size_t fft_scratch_bytes(void* plan);   // scratch slab bytes for one batch
// store_mode 0: collated fft (fft.rs:14-26); 1: rfft upper half (fft.rs:35); 2: natural
// order, unscaled (internal); 3 / 4: 0 / 1 as f32 dB (fft_frames.hpp)
int fft_launch(void* plan, const FftFrames& fr, float2* out, int store_mode, float2* scratch,
               size_t scratch_frames, hipStream_t s);
// sizes that are not powers of two (fft_gen.hip)
void* fftgen_plan_create(int N, int* status);
void fftgen_plan_destroy(void* plan);
size_t fftgen_frame_scratch_bytes(void* plan);
int fftgen_launch(void* plan, const FftFrames& fr, float2* out, int store_mode, float2* scratch,
                  size_t scratch_frames, hipStream_t s);
int stft_carry_launch(const float2* in, long n_in, const float2* hist, float2* hist_next, long H,
                      hipStream_t s);
int stft_carry_u8_launch(const unsigned short* in, long n_in, const float2* hist,
                         float2* hist_next, long H, hipStream_t s);

}  // namespace sdrgpu
