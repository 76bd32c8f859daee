// abi_resample.cpp -- C ABI of the sample-rate converter: the libsamplerate functions
// src/resample.rs binds (src_new / src_process / src_reset / src_clone / src_set_ratio /
// src_get_channels / src_delete / src_strerror / src_get_name / src_get_description /
// src_get_version; call sites src/resample.rs:3-135, 189-196), with libsamplerate's
// argument checks, state and error codes, for the zero-order-hold and linear converters.
//
// Split of the work: the position walk of src_zoh.c / src_linear.c (input_index += 1/ratio,
// fmod_one, in_used += lrint(...)) only involves scalars -- the state, the frame counts and
// the ratios -- never sample values, and it is a serial f64 recurrence whose exact rounding
// the outputs depend on.  It runs here on the host (about 5 ns per output frame; one GPU
// lane would take ~4x longer per step) and produces, per output frame, the left source
// frame and the fraction; the GPU evaluates every sample from that table (resample.hip), so
// the counts are known before anything is enqueued and sdrgpu_src_process_dev does not
// have to wait for the device.  Built with -ffp-contract=off: the walk's f64 arithmetic must
// round like libsamplerate's.
#include <cmath>
#include <cstring>

#include "abi_common.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

namespace sdrgpu {
int src_interp_launch(bool linear, const float* in, long channels, const int* left,
                      const double* frac, long nframes, const float* last_value, float* out,
                      hipStream_t s);
}

namespace {

constexpr double kSrcMaxRatio = 256.0;           // SRC_MAX_RATIO
constexpr double kSrcMinRatioDiff = 1e-20;       // SRC_MIN_RATIO_DIFF

bool is_bad_src_ratio(double r) { return r < 1.0 / kSrcMaxRatio || r > kSrcMaxRatio; }

// src_linear.c / src_zoh.c fmod_one: x - lrint(x), wrapped into [0, 1)
double fmod_one(double x) {
    const double res = x - (double)std::lrint(x);
    return res < 0.0 ? res + 1.0 : res;
}

// Pinned host table of (left frame, fraction) per output frame; two slots so the walk of
// call i+1 can fill one while call i's upload of the other is still in flight.
struct PinnedTable {
    void* ptr = nullptr;
    size_t cap = 0;  // frames
    hipEvent_t done = nullptr;
    bool pending = false;
    int* left() const { return static_cast<int*>(ptr); }
    double* frac() const { return reinterpret_cast<double*>(static_cast<char*>(ptr) + cap * 4); }
    int ensure(size_t frames) {
        if (pending && hipEventSynchronize(done) != hipSuccess) return SDRGPU_ERR_DEVICE;
        pending = false;
        if (frames <= cap) return SDRGPU_OK;
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        cap = 0;
        size_t want = frames < 4096 ? 4096 : frames;
        want = (want + 1) & ~size_t(1);  // keep the f64 half 8-byte aligned
        if (hipHostMalloc(&ptr, want * 12) != hipSuccess) return SDRGPU_ERR_NOMEM;
        cap = want;
        return SDRGPU_OK;
    }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        if (done) (void)hipEventDestroy(done);
        ptr = nullptr;
        done = nullptr;
        cap = 0;
        pending = false;
    }
};

const char* const kNames[5] = {"Best Sinc Interpolator", "Medium Sinc Interpolator",
                               "Fastest Sinc Interpolator", "ZOH Interpolator",
                               "Linear Interpolator"};
const char* const kDescriptions[5] = {
    "Band limited sinc interpolation, best quality, 144dB SNR, 96% BW.",
    "Band limited sinc interpolation, medium quality, 121dB SNR, 90% BW.",
    "Band limited sinc interpolation, fastest, 97dB SNR, 80% BW.",
    "Zero order hold interpolator, very fast, poor quality.",
    "Linear interpolator, very fast, poor quality.",
};

}  // namespace

struct sdrgpu_src_state {
    int device = 0, type = SDRGPU_SRC_LINEAR, channels = 1;
    // SRC_STATE + LINEAR_DATA / ZOH_DATA (host side; last_value lives on the device)
    double last_position = 0.0, last_ratio = 0.0;
    bool reset_pending = true;
    float* d_last_value = nullptr;
    StreamSlot stream;
    PinnedTable table[2];
    int slot = 0;
    DevBuf d_table, stage_in, stage_out;

    bool linear() const { return type == SDRGPU_SRC_LINEAR; }
    void free_all() {
        DeviceGuard g(device);
        if (d_last_value) (void)hipFree(d_last_value);
        d_last_value = nullptr;
        for (auto& t : table) t.release();
        d_table.release();
        stage_in.release();
        stage_out.release();
        stream.destroy();
    }
    int init(int dev, int typ, int ch) {
        device = dev;
        type = typ;
        channels = ch;
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_SRC_ERR_BAD_STATE;
        if (stream.create()) return SDRGPU_SRC_ERR_BAD_STATE;
        if (hipMalloc(&d_last_value, sizeof(float) * (size_t)channels) != hipSuccess)
            return SDRGPU_SRC_ERR_MALLOC_FAILED;
        for (auto& t : table)
            if (hipEventCreateWithFlags(&t.done, hipEventDisableTiming) != hipSuccess)
                return SDRGPU_SRC_ERR_MALLOC_FAILED;
        return reset();
    }
    // src_reset: last_position = last_ratio = 0, converter reset (last_value cleared and
    // re-primed from the next block's first frame)
    int reset() {
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_SRC_ERR_BAD_STATE;
        last_position = 0.0;
        last_ratio = 0.0;
        reset_pending = true;
        if (hipMemsetAsync(d_last_value, 0, sizeof(float) * (size_t)channels, stream.cur) !=
                hipSuccess ||
            hipStreamSynchronize(stream.cur) != hipSuccess)
            return SDRGPU_SRC_ERR_BAD_STATE;
        return 0;
    }

    // The process loop of src_linear.c / src_zoh.c over the scalars only (sample counts
    // in_count / out_count / in_used / out_gen are in SAMPLES = frames x channels, as there).
    // Writes the per-output-frame table and returns the libsamplerate status.
    int walk(const sdrgpu_src_data& d, int* left, double* frac, size_t cap, long* in_used_out,
             long* out_gen_out) {
        const long ch = channels;
        const long in_count = d.input_frames * ch, out_count = d.output_frames * ch;
        long in_used = 0, out_gen = 0;
        size_t k = 0;
        double src_ratio = last_ratio;
        if (is_bad_src_ratio(src_ratio)) return SDRGPU_SRC_ERR_BAD_INTERNAL_STATE;
        const bool vari = std::fabs(last_ratio - d.src_ratio) > kSrcMinRatioDiff;
        double input_index = last_position;
        const bool lin = linear();

        // samples before the first input frame: interpolate from last_value
        while (input_index < 1.0 && out_gen < out_count) {
            const double need = lin ? (double)ch * (1.0 + input_index) : (double)ch * input_index;
            if ((double)in_used + need >= (double)in_count) break;
            if (out_count > 0 && vari)
                src_ratio = last_ratio + (double)out_gen * (d.src_ratio - last_ratio) / (double)out_count;
            if (k >= cap) return SDRGPU_SRC_ERR_BAD_INTERNAL_STATE;
            left[k] = -1;
            frac[k] = input_index;
            ++k;
            out_gen += ch;
            input_index += 1.0 / src_ratio;
        }
        double rem = fmod_one(input_index);
        in_used += ch * std::lrint(input_index - rem);
        input_index = rem;

        // main loop
        for (;;) {
            if (out_gen >= out_count) break;
            const double pos = (double)in_used + (double)ch * input_index;
            if (lin ? !(pos < (double)in_count) : !(pos <= (double)in_count)) break;
            if (out_count > 0 && vari)
                src_ratio = last_ratio + (double)out_gen * (d.src_ratio - last_ratio) / (double)out_count;
            if (k >= cap) return SDRGPU_SRC_ERR_BAD_INTERNAL_STATE;
            left[k] = (int)((in_used - ch) / ch);
            frac[k] = input_index;
            ++k;
            out_gen += ch;
            input_index += 1.0 / src_ratio;
            rem = fmod_one(input_index);
            in_used += ch * std::lrint(input_index - rem);
            input_index = rem;
        }
        if (in_used > in_count) {
            input_index += (double)((in_used - in_count) / ch);
            in_used = in_count;
        }
        last_position = input_index;
        last_ratio = src_ratio;
        *in_used_out = in_used;
        *out_gen_out = out_gen;
        return 0;
    }

    // src_process after its argument checks + the converter; d_in / d_out are device
    // pointers (the host-pointer entry point passes its staging buffers).
    int process(sdrgpu_src_data* user, const float* d_in, float* d_out) {
        sdrgpu_src_data& d = *user;
        d.input_frames_used = 0;
        d.output_frames_gen = 0;
        if (last_ratio < 1.0 / kSrcMaxRatio) last_ratio = d.src_ratio;
        if (d.input_frames <= 0) return 0;
        DeviceGuard g(device);
        if (!g.ok()) return SDRGPU_SRC_ERR_BAD_STATE;
        const size_t fb = sizeof(float) * (size_t)channels;
        if (reset_pending) {  // "If we have just been reset, set the last_value data."
            if (hipMemcpyAsync(d_last_value, d_in, fb, hipMemcpyDeviceToDevice, stream.cur) !=
                hipSuccess)
                return SDRGPU_SRC_ERR_BAD_STATE;
            reset_pending = false;
        }
        // output frames the walk can produce: bounded by the capacity and by the input
        const double rmax = std::fmax(last_ratio, d.src_ratio);
        const double bound = ((double)d.input_frames + 2.0) * rmax + 8.0;
        const size_t nmax = (size_t)std::fmin((double)d.output_frames, bound);
        PinnedTable& t = table[slot];
        if (t.ensure(nmax)) return SDRGPU_SRC_ERR_MALLOC_FAILED;
        long in_used = 0, out_gen = 0;
        int st = walk(d, t.left(), t.frac(), t.cap, &in_used, &out_gen);
        if (st) return st;
        const long nout = out_gen / channels;
        if (nout > 0) {
            // device table: left[nout] (int32), then frac[nout] (f64) at the next 8-byte boundary
            const size_t foff = ((size_t)nout * 4 + 7) & ~size_t(7);
            if (d_table.ensure(foff + (size_t)nout * 8)) return SDRGPU_SRC_ERR_MALLOC_FAILED;
            int* dl = static_cast<int*>(d_table.ptr);
            double* dfr = reinterpret_cast<double*>(static_cast<char*>(d_table.ptr) + foff);
            if (hipMemcpyAsync(dl, t.left(), (size_t)nout * 4, hipMemcpyHostToDevice,
                               stream.cur) != hipSuccess)
                return SDRGPU_SRC_ERR_BAD_STATE;
            if (linear() && hipMemcpyAsync(dfr, t.frac(), (size_t)nout * 8,
                                           hipMemcpyHostToDevice, stream.cur) != hipSuccess)
                return SDRGPU_SRC_ERR_BAD_STATE;
            if (hipEventRecord(t.done, stream.cur) != hipSuccess) return SDRGPU_SRC_ERR_BAD_STATE;
            t.pending = true;
            slot ^= 1;
            if (src_interp_launch(linear(), d_in, channels, dl, dfr, nout, d_last_value, d_out,
                                  stream.cur))
                return SDRGPU_SRC_ERR_BAD_STATE;
        }
        if (in_used > 0 &&
            hipMemcpyAsync(d_last_value, d_in + (in_used - channels), fb,
                           hipMemcpyDeviceToDevice, stream.cur) != hipSuccess)
            return SDRGPU_SRC_ERR_BAD_STATE;
        d.input_frames_used = in_used / channels;
        d.output_frames_gen = nout;
        return 0;
    }
};

namespace {

// src_process's argument checks (samplerate.c), before any state is touched
int check_data(const sdrgpu_src_state* s, sdrgpu_src_data* d) {
    if (!s) return SDRGPU_SRC_ERR_BAD_STATE;
    if (!d) return SDRGPU_SRC_ERR_BAD_DATA;
    if ((!d->data_in && d->input_frames > 0) || (!d->data_out && d->output_frames > 0))
        return SDRGPU_SRC_ERR_BAD_DATA_PTR;
    if (is_bad_src_ratio(d->src_ratio)) return SDRGPU_SRC_ERR_BAD_SRC_RATIO;
    if (d->input_frames < 0) d->input_frames = 0;
    if (d->output_frames < 0) d->output_frames = 0;
    const long ch = s->channels;
    if (d->data_in < d->data_out) {
        if (d->data_in + d->input_frames * ch > d->data_out) return SDRGPU_SRC_ERR_DATA_OVERLAP;
    } else if (d->data_out + d->output_frames * ch > d->data_in) {
        return SDRGPU_SRC_ERR_DATA_OVERLAP;
    }
    if (d->input_frames > (long)INT32_MAX) return SDRGPU_SRC_ERR_BAD_DATA;  // 32-bit frame ids
    return 0;
}

}  // namespace

extern "C" {

sdrgpu_src_state* sdrgpu_src_new(int device, int converter_type, int channels, int* error) {
    int dummy;
    int* err = error ? error : &dummy;
    *err = 0;
    // the sinc converters need libsamplerate's coefficient tables (not in this image)
    if (converter_type < SDRGPU_SRC_ZERO_ORDER_HOLD || converter_type > SDRGPU_SRC_LINEAR) {
        *err = SDRGPU_SRC_ERR_BAD_CONVERTER;
        return nullptr;
    }
    if (channels < 1) {
        *err = SDRGPU_SRC_ERR_BAD_CHANNEL_COUNT;
        return nullptr;
    }
    if (check_device(device)) {
        *err = SDRGPU_SRC_ERR_BAD_STATE;
        return nullptr;
    }
    auto* s = new (std::nothrow) sdrgpu_src_state();
    if (!s) {
        *err = SDRGPU_SRC_ERR_MALLOC_FAILED;
        return nullptr;
    }
    if (int st = s->init(device, converter_type, channels)) {
        s->free_all();
        delete s;
        *err = st;
        return nullptr;
    }
    return s;
}

int sdrgpu_src_process_dev(sdrgpu_src_state* s, sdrgpu_src_data* d) {
    if (int st = check_data(s, d)) return st;
    return s->process(d, d->data_in, d->data_out);
}

int sdrgpu_src_process(sdrgpu_src_state* s, sdrgpu_src_data* d) {
    if (int st = check_data(s, d)) return st;
    DeviceGuard g(s->device);
    if (!g.ok()) return SDRGPU_SRC_ERR_BAD_STATE;
    const size_t fb = sizeof(float) * (size_t)s->channels;
    const size_t nin = d->input_frames > 0 ? (size_t)d->input_frames : 0;
    // staged output: never more frames than the input can produce
    const double rmax = std::fmax(s->last_ratio < 1.0 / kSrcMaxRatio ? d->src_ratio : s->last_ratio,
                                  d->src_ratio);
    const size_t nout_max =
        (size_t)std::fmin((double)d->output_frames, ((double)nin + 2.0) * rmax + 8.0);
    if (s->stage_in.ensure(nin * fb) || s->stage_out.ensure(nout_max * fb))
        return SDRGPU_SRC_ERR_MALLOC_FAILED;
    if (nin && hipMemcpyAsync(s->stage_in.ptr, d->data_in, nin * fb, hipMemcpyHostToDevice,
                              s->stream.cur) != hipSuccess)
        return SDRGPU_SRC_ERR_BAD_STATE;
    float* user_out = d->data_out;
    int st = s->process(d, static_cast<const float*>(s->stage_in.ptr),
                        static_cast<float*>(s->stage_out.ptr));
    if (st) return st;
    if (d->output_frames_gen > 0 &&
        hipMemcpyAsync(user_out, s->stage_out.ptr, (size_t)d->output_frames_gen * fb,
                       hipMemcpyDeviceToHost, s->stream.cur) != hipSuccess)
        return SDRGPU_SRC_ERR_BAD_STATE;
    if (hipStreamSynchronize(s->stream.cur) != hipSuccess) return SDRGPU_SRC_ERR_BAD_STATE;
    return 0;
}

int sdrgpu_src_sync(sdrgpu_src_state* s) {
    if (!s) return SDRGPU_SRC_ERR_BAD_STATE;
    DeviceGuard g(s->device);
    return hipStreamSynchronize(s->stream.cur) == hipSuccess ? 0 : SDRGPU_SRC_ERR_BAD_STATE;
}

int sdrgpu_src_reset(sdrgpu_src_state* s) {
    if (!s) return SDRGPU_SRC_ERR_BAD_STATE;
    return s->reset();
}

sdrgpu_src_state* sdrgpu_src_clone(sdrgpu_src_state* s, int* error) {
    int dummy;
    int* err = error ? error : &dummy;
    *err = 0;
    if (!s) {
        *err = SDRGPU_SRC_ERR_BAD_STATE;
        return nullptr;
    }
    sdrgpu_src_state* c = sdrgpu_src_new(s->device, s->type, s->channels, err);
    if (!c) return nullptr;
    c->last_position = s->last_position;
    c->last_ratio = s->last_ratio;
    c->reset_pending = s->reset_pending;
    DeviceGuard g(s->device);
    if (hipMemcpyAsync(c->d_last_value, s->d_last_value, sizeof(float) * (size_t)s->channels,
                       hipMemcpyDeviceToDevice, s->stream.cur) != hipSuccess ||
        hipStreamSynchronize(s->stream.cur) != hipSuccess) {
        c->free_all();
        delete c;
        *err = SDRGPU_SRC_ERR_BAD_STATE;
        return nullptr;
    }
    return c;
}

int sdrgpu_src_get_channels(sdrgpu_src_state* s) {
    return s ? s->channels : -SDRGPU_SRC_ERR_BAD_STATE;
}

int sdrgpu_src_set_ratio(sdrgpu_src_state* s, double new_ratio) {
    if (!s) return SDRGPU_SRC_ERR_BAD_STATE;
    if (is_bad_src_ratio(new_ratio)) return SDRGPU_SRC_ERR_BAD_SRC_RATIO;
    s->last_ratio = new_ratio;
    return 0;
}

int sdrgpu_src_set_stream(sdrgpu_src_state* s, void* hip_stream) {
    if (!s) return SDRGPU_SRC_ERR_BAD_STATE;
    s->stream.set(hip_stream);
    return 0;
}

int sdrgpu_src_get_stream(sdrgpu_src_state* s, void** hip_stream) {
    if (!s || !hip_stream) return SDRGPU_SRC_ERR_BAD_STATE;
    *hip_stream = s->stream.cur;
    return 0;
}

sdrgpu_src_state* sdrgpu_src_delete(sdrgpu_src_state* s) {
    if (s) {
        (void)sdrgpu_src_sync(s);
        s->free_all();
        delete s;
    }
    return nullptr;
}

const char* sdrgpu_src_strerror(int error) {
    switch (error) {
        case 0: return "No error.";
        case 1: return "Malloc failed.";
        case 2: return "SRC_STATE pointer is NULL.";
        case 3: return "SRC_DATA pointer is NULL.";
        case 4: return "SRC_DATA->data_out or SRC_DATA->data_in is NULL.";
        case 5: return "Internal error. No private data.";
        case 6: return "SRC ratio outside [1/256, 256] range.";
        case 7: return "Internal error. Bad process pointer.";
        case 8: return "Internal error. SHIFT_BITS too large.";
        case 9: return "Internal error. Filter length too large.";
        case 10: return "Bad converter number.";
        case 11: return "Channel count must be >= 1.";
        case 12: return "Internal error. Bad buffer length. Please report this.";
        case 13: return "Internal error. Input data / internal buffer size difference. Please report this.";
        case 14: return "Internal error. Private pointer is NULL. Please report this.";
        case 15: return "Internal error. Bad sinc state.";
        case 16: return "Input and output data arrays overlap.";
        case 17: return "Supplied callback function pointer is NULL.";
        case 18: return "Calling mode differs from initialisation mode (ie process v callback).";
        case 19: return "Callback function pointer is NULL in src_callback_read ().";
        case 20: return "This converter only allows constant conversion ratios.";
        case 21: return "Internal error : Bad length in prepare_data ().";
        case 22: return "Error : Someone is trampling on my internal state.";
        default: return nullptr;
    }
}

const char* sdrgpu_src_get_name(int converter_type) {
    return converter_type >= 0 && converter_type <= 4 ? kNames[converter_type] : nullptr;
}

const char* sdrgpu_src_get_description(int converter_type) {
    return converter_type >= 0 && converter_type <= 4 ? kDescriptions[converter_type] : nullptr;
}

const char* sdrgpu_src_get_version(void) {
    return "sdrgpu-src 1 (libsamplerate ZOH/linear process loops, gfx950)";
}

}  // extern "C"
