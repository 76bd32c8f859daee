// abi_stubs.cpp -- entry points not yet implemented in this build.
#include "abi_common.hpp"

extern "C" {
int sdrgpu_fft_plan(int, size_t, sdrgpu_fft** out) { if (out) *out = nullptr; return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_fft_set_stream(sdrgpu_fft*, void*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_fft_exec(sdrgpu_fft*, const void*, void*, size_t) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_fft_exec_dev(sdrgpu_fft*, const void*, void*, size_t) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_rfft_exec(sdrgpu_fft*, const float*, void*, size_t) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_fft_get_stream(const sdrgpu_fft*, void**) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_get_stream(const sdrgpu_stft*, void**) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_get_stream(const sdrgpu_pll*, void**) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_fft_sync(sdrgpu_fft*) { return SDRGPU_ERR_UNSUPPORTED; }
void sdrgpu_fft_destroy(sdrgpu_fft*) {}
int sdrgpu_fft_freqs(size_t, float, float*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_create(int, size_t, size_t, sdrgpu_stft** out) { if (out) *out = nullptr; return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_set_stream(sdrgpu_stft*, void*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_output_len(const sdrgpu_stft*, size_t, size_t*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_process(sdrgpu_stft*, const void*, size_t, void*, size_t, size_t*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_process_dev(sdrgpu_stft*, const void*, size_t, void*, size_t, size_t*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_sync(sdrgpu_stft*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_stft_reset(sdrgpu_stft*) { return SDRGPU_ERR_UNSUPPORTED; }
void sdrgpu_stft_destroy(sdrgpu_stft*) {}
int sdrgpu_pll_create(int, const sdrgpu_pll_params*, size_t, sdrgpu_pll** out) { if (out) *out = nullptr; return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_set_stream(sdrgpu_pll*, void*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_process(sdrgpu_pll*, const void*, size_t, size_t, float*, uint8_t*, size_t) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_process_dev(sdrgpu_pll*, const void*, size_t, size_t, float*, uint8_t*, size_t) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_state(sdrgpu_pll*, size_t, float*, float*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_sync(sdrgpu_pll*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_reset(sdrgpu_pll*) { return SDRGPU_ERR_UNSUPPORTED; }
int sdrgpu_pll_clone(const sdrgpu_pll*, sdrgpu_pll** out) { if (out) *out = nullptr; return SDRGPU_ERR_UNSUPPORTED; }
void sdrgpu_pll_destroy(sdrgpu_pll*) {}
}
