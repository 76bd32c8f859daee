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
#include <vector>

#include "abi_common.hpp"

using namespace sdrgpu;
using namespace sdrgpu::detail;

#include "resample_kernels.hpp"

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

// Pinned host staging for the per-output-frame sinc descriptors (two slots, as above).
struct PinnedBytes {
    void* ptr = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
    int ensure(size_t bytes) {
        if (pending && hipEventSynchronize(done) != hipSuccess) return SDRGPU_ERR_DEVICE;
        pending = false;
        if (bytes <= cap) return SDRGPU_OK;
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        cap = 0;
        const size_t want = bytes < (1u << 16) ? (1u << 16) : bytes + bytes / 2;
        if (hipHostMalloc(&ptr, want) != hipSuccess) return SDRGPU_ERR_NOMEM;
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

// Sinc coefficient tables.  libsamplerate's own (fastest_coeffs.h, mid_qual_coeffs.h,
// high_qual_coeffs.h) are not in this image; these keep their increments and lengths and
// are Kaiser-windowed sincs designed for the attenuation the converter descriptions quote
// (97 / 121 / 144 dB over the window length, stopband edge at Nyquist), scaled so the
// integer-spaced taps sum to 1.  Same formula and operation order as the oracle's
// oracle_sinc_table (tests/test_resample.py checks the two tables are identical).
struct SincSpec {
    int inc, len;
    double atten_db;
};
constexpr SincSpec kSincSpec[3] = {{2381, 340239, 144.0}, {491, 22438, 121.0}, {128, 2464, 97.0}};

double bessel_i0(double x) {
    double sum = 1.0, term = 1.0;
    const double q = 0.25 * x * x;
    for (int k = 1; k < 500; k++) {
        term *= q / ((double)k * (double)k);
        sum += term;
        if (term < 1e-17 * sum) break;
    }
    return sum;
}

void sinc_table(int conv, std::vector<float>& out) {
    const int inc = kSincSpec[conv].inc, len = kSincSpec[conv].len;
    const double A = kSincSpec[conv].atten_db;
    const double T = (double)(len - 2) / (double)inc;
    const double dw = (A - 8.0) / (2.285 * 2.0 * T);
    const double fc = 1.0 - dw / (2.0 * M_PI);
    const double beta = 0.1102 * (A - 8.7), i0b = bessel_i0(beta);
    std::vector<double> h((size_t)len);
    for (int i = 0; i < len; i++) {
        const double t = (double)i / (double)inc;
        if (t >= T) {
            h[i] = 0.0;
            continue;
        }
        const double x = t / T;
        const double w = bessel_i0(beta * std::sqrt(1.0 - x * x)) / i0b;
        const double sv = i == 0 ? fc : std::sin(M_PI * fc * t) / (M_PI * t);
        h[i] = sv * w;
    }
    double g = h[0];
    for (int i = inc; i < len; i += inc) g += 2.0 * h[i];
    out.resize((size_t)len);
    for (int i = 0; i < len; i++) out[i] = (float)(h[i] / g);
}

constexpr int kShiftBits = 12;            // SHIFT_BITS
constexpr double kFpOne = 4096.0;         // FP_ONE

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

    // sinc converters: src_sinc.c's SINC_FILTER bookkeeping (in samples = frames x
    // channels, as there) on the host; the samples its buffer would hold live in a device
    // WINDOW of the stream (sample w of the window = stream-window sample vlo + w; buffer
    // index i holds window sample voff + i; vend = samples appended so far).
    int coeff_half_len = 0, index_inc = 0, b_len = 0;
    int b_current = 0, b_end = 0, b_real_end = -1;
    long voff = 0, vend = 0, vlo = 0;
    DevBuf win[2], d_coeffs, d_desc;
    int wcur = 0;
    PinnedBytes desc_host[2];
    struct Append {
        long wpos, src, len;  // window position, input sample offset (-1 = zeros), samples
    };
    std::vector<Append> appends;

    bool linear() const { return type == SDRGPU_SRC_LINEAR; }
    bool sinc() const { return type <= SDRGPU_SRC_SINC_FASTEST; }
    void free_all() {
        DeviceGuard g(device);
        if (d_last_value) (void)hipFree(d_last_value);
        d_last_value = nullptr;
        for (auto& t : desc_host) t.release();
        for (auto& w : win) w.release();
        d_coeffs.release();
        d_desc.release();
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
        for (auto& t : desc_host)
            if (hipEventCreateWithFlags(&t.done, hipEventDisableTiming) != hipSuccess)
                return SDRGPU_SRC_ERR_MALLOC_FAILED;
        if (sinc()) {  // sinc_set_converter
            std::vector<float> c;
            sinc_table(type, c);
            coeff_half_len = (int)c.size() - 2;  // ARRAY_LEN (coeffs) - 2
            index_inc = kSincSpec[type].inc;
            int bl = 3 * (int)std::lrint((coeff_half_len + 2.0) / index_inc * kSrcMaxRatio + 1);
            if (bl < 4096) bl = 4096;
            // libsamplerate keeps buffer indices in int; so does the device window
            if ((long)bl * channels + 1 > (long)(INT32_MAX / 4)) return SDRGPU_SRC_ERR_MALLOC_FAILED;
            b_len = bl * channels + 1;
            if (d_coeffs.ensure(c.size() * sizeof(float)) ||
                hipMemcpy(d_coeffs.ptr, c.data(), c.size() * sizeof(float),
                          hipMemcpyHostToDevice) != hipSuccess)
                return SDRGPU_SRC_ERR_MALLOC_FAILED;
        }
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
        b_current = b_end = 0;  // sinc_reset
        b_real_end = -1;
        voff = vend = vlo = 0;
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

    // Output frames one call can produce: bounded by the capacity and by the input plus
    // what the converter holds back (the sinc buffer).
    size_t max_out_frames(const sdrgpu_src_data& d) const {
        const double r0 = last_ratio < 1.0 / kSrcMaxRatio ? d.src_ratio : last_ratio;
        const double rmax = std::fmax(r0, d.src_ratio);
        double in = (double)(d.input_frames > 0 ? d.input_frames : 0) + 2.0;
        if (sinc()) in += (double)b_len / channels;
        return (size_t)std::fmin((double)(d.output_frames > 0 ? d.output_frames : 0),
                                 in * rmax + 8.0);
    }

    // window room for this call: compact to the live samples [voff, vend) when needed
    int sinc_window(long need_more) {
        const long live = vend - voff;
        const size_t need = (size_t)(vend - vlo + need_more) * sizeof(float);
        if (need <= win[wcur].cap) return 0;
        const size_t want = (size_t)(live + need_more) * 2 * sizeof(float);
        DevBuf& dst = win[wcur ^ 1];
        if (dst.cap < want) {
            if (hipStreamSynchronize(stream.cur) != hipSuccess) return SDRGPU_SRC_ERR_BAD_STATE;
            if (dst.ensure(want)) return SDRGPU_SRC_ERR_MALLOC_FAILED;
        }
        if (live > 0 &&
            hipMemcpyAsync(dst.ptr, static_cast<float*>(win[wcur].ptr) + (voff - vlo),
                           (size_t)live * sizeof(float), hipMemcpyDeviceToDevice,
                           stream.cur) != hipSuccess)
            return SDRGPU_SRC_ERR_BAD_STATE;
        wcur ^= 1;
        vlo = voff;
        return 0;
    }

    // buffer samples [b_end, b_end + len) become input samples [src, src + len) (src = -1:
    // zeros) -- libsamplerate's memcpy / memset into its buffer
    int sinc_append(long src, long len) {
        if (vend != voff + b_end) return SDRGPU_SRC_ERR_BAD_INTERNAL_STATE;
        if (len > 0) appends.push_back({vend - vlo, src, len});
        vend += len;
        b_end += (int)len;
        return 0;
    }

    // src_sinc.c prepare_data over the bookkeeping only
    int sinc_prepare(long in_count, long* in_used, bool in_null, bool eoi, int half) {
        const int ch = channels;
        int len = 0;
        if (b_real_end >= 0) return 0;
        if (in_null) return 0;
        if (b_current == 0) {
            len = b_len - 2 * half;
            b_end = 0;  // the lead-in zeros [0, half) of the reset buffer
            if (int st = sinc_append(-1, half)) return st;
            b_current = half;
        } else if (b_end + half + ch < b_len) {
            len = std::max(b_len - b_current - half, 0);
        } else {
            len = b_end - b_current;
            if (b_current - half < 0) return SDRGPU_SRC_ERR_SINC_PREPARE_DATA_BAD_LEN;
            voff += b_current - half;  // memmove (buffer, buffer + b_current - half, ...)
            b_current = half;
            b_end = b_current + len;
            len = std::max(b_len - b_current - half, 0);
        }
        if ((long)len > in_count - *in_used) len = (int)(in_count - *in_used);
        len -= len % ch;
        if (len < 0 || b_end + len > b_len) return SDRGPU_SRC_ERR_SINC_PREPARE_DATA_BAD_LEN;
        if (int st = sinc_append(*in_used, len)) return st;
        *in_used += len;
        if (*in_used == in_count && b_end - b_current < 2 * half && eoi) {
            if (b_len - b_end < half + 5) {
                len = b_end - b_current;
                if (b_current - half < 0) return SDRGPU_SRC_ERR_SINC_PREPARE_DATA_BAD_LEN;
                voff += b_current - half;
                b_current = half;
                b_end = b_current + len;
            }
            b_real_end = b_end;
            len = half + 5;
            if (len < 0 || b_end + len > b_len) len = b_len - b_end;
            if (int st = sinc_append(-1, len)) return st;
        }
        return 0;
    }

    // the buffer fills recorded by sinc_append, in order: input copies and zero runs
    int flush_appends(const float* d_in) {
        float* w = static_cast<float*>(win[wcur].ptr);
        for (const Append& a : appends) {
            hipError_t e = a.src < 0
                ? hipMemsetAsync(w + a.wpos, 0, (size_t)a.len * sizeof(float), stream.cur)
                : hipMemcpyAsync(w + a.wpos, d_in + a.src, (size_t)a.len * sizeof(float),
                                 hipMemcpyDeviceToDevice, stream.cur);
            if (e != hipSuccess) return SDRGPU_SRC_ERR_BAD_STATE;
        }
        appends.clear();
        return 0;
    }

    // src_sinc.c's multichannel vari process loop; per output frame a descriptor of
    // calc_output_multi's taps (the samples are summed on the GPU, resample.hip)
    int sinc_process(sdrgpu_src_data& d, const float* d_in, bool in_null, float* d_out) {
        const int ch = channels;
        const long in_count = d.input_frames * ch, out_count = d.output_frames * ch;
        long in_used = 0, out_gen = 0;
        double src_ratio = last_ratio;
        if (is_bad_src_ratio(src_ratio)) return SDRGPU_SRC_ERR_BAD_INTERNAL_STATE;
        double count = (coeff_half_len + 2.0) / index_inc;
        const double rmin = std::fmin(last_ratio, d.src_ratio);
        if (rmin < 1.0) count /= rmin;
        const int half = ch * ((int)std::lrint(count) + 1);
        double input_index = last_position;
        double rem = fmod_one(input_index);
        b_current = (b_current + ch * (int)std::lrint(input_index - rem)) % b_len;
        input_index = rem;
        const double terminate = 1.0 / src_ratio + 1e-20;
        const bool eoi = d.end_of_input != 0;
        appends.clear();
        // this call appends at most its input, the lead-in zeros and the end-of-input tail
        // (2 half + 5 <= b_len); window indices are int
        if (in_count + 2L * b_len > (long)(INT32_MAX / 2)) return SDRGPU_SRC_ERR_BAD_DATA;
        if (int st = sinc_window(in_count + (long)b_len + 16)) return st;
        const size_t cap_frames = max_out_frames(d);
        PinnedBytes& hb = desc_host[slot];
        if (hb.ensure(cap_frames * sizeof(SincDesc) + sizeof(SincDesc)))
            return SDRGPU_SRC_ERR_MALLOC_FAILED;
        SincDesc* desc = static_cast<SincDesc*>(hb.ptr);
        const int max_fi = coeff_half_len << kShiftBits;
        long k = 0;
        // an error inside the loop leaves the buffer bookkeeping where prepare_data moved it
        // (as libsamplerate, which has already copied the data by then): enqueue the appends
        // recorded so far so the device window matches that bookkeeping before returning
        auto fail = [&](int st) {
            (void)flush_appends(d_in);
            return st;
        };
        while (out_gen < out_count) {
            int in_hand = (b_end - b_current + b_len) % b_len;
            if (in_hand <= half) {
                if (int st = sinc_prepare(in_count, &in_used, in_null, eoi, half)) return fail(st);
                in_hand = (b_end - b_current + b_len) % b_len;
                if (in_hand <= half) break;
            }
            if (b_real_end >= 0 && b_current + input_index + terminate > b_real_end) break;
            if (out_count > 0 && std::fabs(last_ratio - d.src_ratio) > 1e-10)
                src_ratio = last_ratio + (double)out_gen * (d.src_ratio - last_ratio) / (double)out_count;
            const double float_increment = index_inc * (src_ratio < 1.0 ? src_ratio : 1.0);
            const int inc = (int)std::lrint(float_increment * kFpOne);
            const int start = (int)std::lrint(input_index * float_increment * kFpOne);
            if ((size_t)k >= cap_frames) return fail(SDRGPU_SRC_ERR_BAD_INTERNAL_STATE);
            SincDesc& o = desc[k++];
            // left half (with the underflow skip of calc_output_multi)
            int fi = start;
            int cc = (max_fi - fi) / inc;
            fi += cc * inc;
            int di = b_current - ch * cc;
            if (di < 0) {
                const int steps = (-di + ch - 1) / ch;
                fi -= inc * steps;
                di += steps * ch;
            }
            o.fil = fi;
            o.nl = fi >= 0 ? fi / inc + 1 : 0;
            o.dl = (int)(voff + di - vlo);
            // right half (do-while: at least one tap)
            fi = inc - start;
            cc = (max_fi - fi) / inc;
            fi += cc * inc;
            o.fir = fi;
            o.nr = fi > 0 ? (fi + inc - 1) / inc : 1;
            o.dr = (int)(voff + b_current + ch * (1 + cc) - vlo);
            o.inc = inc;
            o.pad = 0;
            o.scale = float_increment / index_inc;
            out_gen += ch;
            input_index += 1.0 / src_ratio;
            rem = fmod_one(input_index);
            b_current = (b_current + ch * (int)std::lrint(input_index - rem)) % b_len;
            input_index = rem;
        }
        last_position = input_index;
        last_ratio = src_ratio;
        // enqueue: the buffer fills (input copies / zeros), the descriptors, the sums
        if (int st = flush_appends(d_in)) return st;
        float* w = static_cast<float*>(win[wcur].ptr);
        if (k > 0) {
            if (d_desc.ensure((size_t)k * sizeof(SincDesc))) return SDRGPU_SRC_ERR_MALLOC_FAILED;
            if (hipMemcpyAsync(d_desc.ptr, desc, (size_t)k * sizeof(SincDesc),
                               hipMemcpyHostToDevice, stream.cur) != hipSuccess ||
                hipEventRecord(hb.done, stream.cur) != hipSuccess)
                return SDRGPU_SRC_ERR_BAD_STATE;
            hb.pending = true;
            slot ^= 1;
            if (src_sinc_launch(w, ch, static_cast<const SincDesc*>(d_desc.ptr), k,
                                static_cast<const float*>(d_coeffs.ptr), coeff_half_len + 2, d_out,
                                stream.cur))
                return SDRGPU_SRC_ERR_BAD_STATE;
        }
        d.input_frames_used = in_used / ch;
        d.output_frames_gen = k;
        return 0;
    }

    // src_process after its argument checks + the converter; d_in / d_out are device
    // pointers (the host-pointer entry point passes its staging buffers).
    int process(sdrgpu_src_data* user, const float* d_in, float* d_out, bool in_null) {
        sdrgpu_src_data& d = *user;
        d.input_frames_used = 0;
        d.output_frames_gen = 0;
        if (last_ratio < 1.0 / kSrcMaxRatio) last_ratio = d.src_ratio;
        if (sinc()) {
            DeviceGuard g(device);
            if (!g.ok()) return SDRGPU_SRC_ERR_BAD_STATE;
            return sinc_process(d, d_in, in_null, d_out);
        }
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
        const size_t nmax = max_out_frames(d);
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
    if (converter_type < SDRGPU_SRC_SINC_BEST_QUALITY || converter_type > SDRGPU_SRC_LINEAR) {
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
    return s->process(d, d->data_in, d->data_out, d->data_in == nullptr);
}

int sdrgpu_src_process(sdrgpu_src_state* s, sdrgpu_src_data* d) {
    if (int st = check_data(s, d)) return st;
    DeviceGuard g(s->device);
    if (!g.ok()) return SDRGPU_SRC_ERR_BAD_STATE;
    const size_t fb = sizeof(float) * (size_t)s->channels;
    const size_t nin = d->input_frames > 0 ? (size_t)d->input_frames : 0;
    // staged output: never more frames than the call can produce
    const size_t nout_max = s->max_out_frames(*d);
    if (s->stage_in.ensure(nin * fb) || s->stage_out.ensure(nout_max * fb))
        return SDRGPU_SRC_ERR_MALLOC_FAILED;
    if (nin && hipMemcpyAsync(s->stage_in.ptr, d->data_in, nin * fb, hipMemcpyHostToDevice,
                              s->stream.cur) != hipSuccess)
        return SDRGPU_SRC_ERR_BAD_STATE;
    float* user_out = d->data_out;
    int st = s->process(d, static_cast<const float*>(s->stage_in.ptr),
                        static_cast<float*>(s->stage_out.ptr), d->data_in == nullptr);
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
    if (s->sinc()) {  // the buffer bookkeeping and the live window samples
        c->b_current = s->b_current;
        c->b_end = s->b_end;
        c->b_real_end = s->b_real_end;
        c->voff = s->voff;
        c->vend = s->vend;
        c->vlo = s->voff;
        c->wcur = 0;
        const long live = s->vend - s->voff;
        if (c->win[0].ensure((size_t)(live > 0 ? live : 1) * 2 * sizeof(float)) ||
            (live > 0 &&
             hipMemcpyAsync(c->win[0].ptr, static_cast<float*>(s->win[s->wcur].ptr) + (s->voff - s->vlo),
                            (size_t)live * sizeof(float), hipMemcpyDeviceToDevice,
                            s->stream.cur) != hipSuccess)) {
            c->free_all();
            delete c;
            *err = SDRGPU_SRC_ERR_BAD_STATE;
            return nullptr;
        }
    }
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
    return "sdrgpu-src 2 (libsamplerate sinc/ZOH/linear process loops, own sinc tables, gfx950)";
}

int sdrgpu_src_sinc_table(int converter_type, float* coeffs, int cap, int* increment) {
    if (converter_type < SDRGPU_SRC_SINC_BEST_QUALITY || converter_type > SDRGPU_SRC_SINC_FASTEST)
        return -1;
    if (increment) *increment = kSincSpec[converter_type].inc;
    const int len = kSincSpec[converter_type].len;
    if (!coeffs) return len;
    if (cap < len) return -1;
    std::vector<float> c;
    sinc_table(converter_type, c);
    std::memcpy(coeffs, c.data(), c.size() * sizeof(float));
    return len;
}

}  // extern "C"
