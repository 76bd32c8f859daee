// fft64k_xcd.hip -- EXPERIMENT, not built into libsdrgpu.so (round 3, measured and dropped).
//
// configs[2]'s 64 Ki-point four-step as ONE persistent launch that keeps every frame's pass-A
// -> pass-B hand-off inside one XCD's L2 (the round-2 verdict's "XCD-resident schedule").  The
// kernel excerpt below dropped into unnamed-rust-sdr_amd/csrc/fft.hip ahead of the dif4 kernel,
// and the launch block into fft_launch() ahead of the two-launch 64K path (it reads the
// SDRGPU_F64X* tuning variables listed there).  Parity: the 64K STFT tests of
// tests/test_fft_gpu.py (700-frame multi-batch c64 / dB / u8, 1-64-frame edge cases, six
// back-to-back runs bit-identical) were green on it, with no spin timeout.
//
// Measured (bench_configs.py --config c3, 2^28 c64 samples, 8192 frames; profiles/
// r03_c3_xcd_experiment.txt): 3.06-4.3 ms over ring sizes 2-8, lags 1-6, 1 / 2 / 4
// workgroups per CU, chunks 1-16, plain / nt input, nt / sc1 output -- against 2.52-2.54 ms for
// the two-launch path on the same boxes.  PMC (FETCH x2 + WRITE): with one workgroup per CU
// and a 4-frame ring the scratch reads DO hit the XCD's L2 (FETCH 6.7 -> 2.5 GB per step), but
// WRITE_SIZE stays 8.6 GB: every store leaves the L2 (write-through for these stores on
// gfx950), so the 4.3 GB of scratch writes reach the fabric whatever the schedule, and the
// floor of any two-pass 64K form is input + scratch writes + output = 1.67x algorithmic.
// Ablations (timing only, wrong results): no dependency waits 3.40-3.53 ms, no store drain
// before the hand-off counter no change -- the launch is slow per piece (67 % of wave time
// waiting on memory, 2 workgroups of 8 waves per CU), not on its synchronisation.

// ---- kernel excerpt (namespace sdrgpu, anonymous namespace of fft.hip) ----
// -------- 65536-point four-step as ONE persistent launch with XCD-resident scratch ----------
// The two-launch form above sends every pass-A result (512 KiB per frame) out through the
// fabric to the MALL/HBM slab and back: 2.4x the algorithmic bytes.  Here the same two pieces
// of work -- A(f, blk): FFT-256 down CB columns of frame f into the scratch; B(f, blk): FFT-256
// along CB rows of it into the output -- are dealt from a ticket counter PER XCD (the XCD id
// read from HW_REG_XCC_ID), and every frame's A and B pieces run on the CUs of ONE XCD through
// a small ring of NS scratch frames of that XCD, so the hand-off stays in its 4 MiB L2.
// Correctness does not depend on placement: a piece only ever waits for pieces with LOWER
// tickets of its own queue (B(s) on A(s); A(s) on B(s - NS) freeing its scratch frame; a
// slot's frame id on the slot's first A ticket), each held by a running workgroup, and the
// producer and consumer of a hand-off read the same XCC id, so they share the L2 (plain
// stores acknowledged by the L2 -> counter; L1-bypassing loads on the consumer).  Frames are
// claimed per XCD in chunks of C consecutive frames, so a frame's first half (the previous
// frame's second half at hop N/2) is still in the same L2.  Every spin is bounded; a timeout
// sets ctl word kFault (checked by the tests) and the launch still drains.
namespace xr {
constexpr int kXcd = 8;
constexpr int kPubRing = 64;           // slot -> frame id publication ring (tagged by slot)
constexpr int kXWords = 1024;          // control words per XCD (4 KiB)
constexpr int kCtlWords = 64 + kXcd * kXWords;
constexpr size_t kCtlBytes = 64 << 10; // control block at the start of the scratch slab
constexpr int kFault = 32;             // global word: spin timeouts
constexpr int kNsMax = 8;
// per-XCD words: [0] ticket, [32 (1 + i)] A pieces done on ring frame i (cumulative),
// [32 (9 + i)] B pieces done on ring frame i (cumulative), [544 ...] pub ring (u64)
__device__ __forceinline__ unsigned* a_cnt(unsigned* X, int i) { return X + 32 * (1 + i); }
__device__ __forceinline__ unsigned* b_cnt(unsigned* X, int i) { return X + 32 * (9 + i); }
__device__ __forceinline__ unsigned long long* pub(unsigned* X, unsigned s) {
    return reinterpret_cast<unsigned long long*>(X + 544) + (s % kPubRing);
}
__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kSpin = 1 << 18;
__device__ __forceinline__ bool spin_ge(const unsigned* p, unsigned target, unsigned* fault) {
    for (int it = 0; it < kSpin; ++it) {
        if (ld_agent(p) >= target) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    atomicOr(fault, 1u);
    return false;
}
constexpr long kEmpty = 1L << 40;
// frame id published for slot s (tag s + 1 in the high word); kEmpty on timeout
__device__ __forceinline__ long wait_pub(unsigned* X, unsigned s, unsigned* fault) {
    unsigned long long* p = pub(X, s);
    for (int it = 0; it < kSpin; ++it) {
        const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(v >> 32) == s + 1) return (long)(v & 0xffffffffull);
        __builtin_amdgcn_s_sleep(1);
    }
    atomicOr(fault, 2u);
    return kEmpty;
}
__device__ __forceinline__ void publish(unsigned* X, unsigned s, long fid) {
    const unsigned long long v = ((unsigned long long)(s + 1) << 32) |
                                 (unsigned long long)(fid > 0xfffffff0L ? 0xfffffff0L : fid);
    __hip_atomic_store(pub(X, s), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace xr

struct F64XArgs {
    F64Args f;
    unsigned* ctl;   // kCtlWords, zeroed before the launch
    float2* ring;    // kXcd x NS frames of scratch
    int ns;          // scratch frames per XCD (2..kNsMax)
    int chunk;       // consecutive frames claimed per XCD at a time
    int nowait;      // TEMP ablation
    int inpol, outpol, nodrain;  // TEMP
    int lag;         // B pieces of slot s ride on the tickets of slot s + lag (1 <= lag < ns)
};

// A(f, blk): pass A of fft64k_pass_a for columns CB*blk .. +CB of frame f, into S
template <int CB>
__device__ __forceinline__ void f64_piece_a(const F64Args& a, long f, int blk, float2* lds, float2* S,
                                            int inpol) {
    constexpr long M = 65536;
    const int c = threadIdx.x % CB, j = threadIdx.x / CB;
    const int col = CB * blk + c;
    float2 v[16];
    const FrameSrc& s = a.src;
    long g0 = 0;
    bool fast = s.mode == 0;
    if (s.mode == 1) {
        g0 = s.first_end + f * s.hop - M;
        fast = g0 >= 0 && g0 + M <= s.n_in;
    }
    if (fast) {
        const float2* src = s.mode == 0 ? s.in + f * M : s.in + g0;
        if (inpol == 1) {
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = ld_nt(src + 256 * (j + 16 * m) + col);
        } else {
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = src[256 * (j + 16 * m) + col];
        }
    } else {
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = frame_sample(s, M, f, 256 * (j + 16 * m) + col);
    }
    Dft<16, false>::run(v);
    if (j) twiddle<16, false>(v, a.tw, 16 * j);
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) lds[(ka * 16 + j) * CB + c] = v[ka];
    __syncthreads();
    const int ka = j;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = lds[(ka * 16 + jj) * CB + c];
    Dft<16, false>::run(v);
    const float2 w1 = a.twM[col * ka];
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) v[kb] = cmul(v[kb], w1);
    twiddle<16, false>(v, a.tw, col);
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) S[(ka + 16 * kb) * 256 + col] = v[kb];
}

// B(f, blk): pass B of fft64k_pass_b for rows k1 = CB*blk .. +CB of S into frame f's output;
// `release` runs once every wave's scratch loads have landed (after the first LDS barrier)
template <int CB, typename Rel>
__device__ __forceinline__ void f64_piece_b(const F64Args& a, long f, int blk, float2* lds,
                                            const float2* S, const Rel& release, int outpol) {
    constexpr int P = CB + 1;
    constexpr long M = 65536;
    constexpr int NTH = 16 * CB;
    const int t = threadIdx.x;
    const int k1b = CB * blk;
    const float2* Sr = S + k1b * 256;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int p = t + NTH * i;
        lds[(p & 255) * P + (p >> 8)] = ld_nt(Sr + p);  // L1-bypassing: written by other CUs
    }
    __syncthreads();
    release();
    const int r = t % CB, j = t / CB;
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = lds[(j + 16 * m) * P + r];
    __syncthreads();
    Dft<16, false>::run(v);
    if (j) twiddle<16, false>(v, a.tw, 16 * j);
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) lds[(ka * 16 + j) * P + r] = v[ka];
    __syncthreads();
    const int ka = j;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = lds[(ka * 16 + jj) * P + r];
    Dft<16, false>::run(v);
    if (a.store_mode != 0) {
#pragma unroll
        for (int kb = 0; kb < 16; ++kb)
            store_bin(a.out, f, M, (long)(k1b + r) + 256L * (ka + 16 * kb), v[kb], a.store_mode, a.norm);
        return;
    }
    float2* O = a.out + f * M;
    const float nrm = a.norm;
    if (outpol == 1) {
#pragma unroll
        for (int kb = 0; kb < 16; ++kb) {
            const int k2 = (ka + 16 * kb + 128) & 255;
            const float2 y = make_float2(v[kb].x * nrm, v[kb].y * nrm);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(O + (long)k2 * 256 + k1b + r),
                               __builtin_bit_cast(unsigned long long, y), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
        const int k2 = (ka + 16 * kb + 128) & 255;
        st_nt(O + (long)k2 * 256 + k1b + r, make_float2(v[kb].x * nrm, v[kb].y * nrm));
    }
}

// Lane 0 of wave 0 is the workgroup's scheduler.  It holds two drawn tickets beyond the one in
// work, and at the start of every piece issues the loads the NEXT ticket's resolution needs
// (its slot's publication word and the counter it waits on), so at the end of the piece those
// values are normally already there and satisfied: no poll round trip between pieces.
struct XPre {
    unsigned long long pub;  // prefetched publication word (tag checked on use)
    unsigned cnt;            // prefetched dependency counter
};

template <int CB>
__global__ __launch_bounds__(16 * CB, 4) void fft64k_xcd_kernel(F64XArgs a) {
    constexpr int PPF = 256 / CB;                 // A (and B) pieces per frame
    constexpr unsigned TPS = 2 * PPF;             // tickets per slot
    constexpr int LDSN = 256 * (CB + 1);          // >= 16 * 16 * CB
    constexpr unsigned kHwXcc = 20u | (3u << 11);  // hwreg(HW_REG_XCC_ID, 0, 4)
    __shared__ float2 lds[LDSN];
    __shared__ long desc[2];
    const unsigned x = __builtin_amdgcn_s_getreg(kHwXcc) & (xr::kXcd - 1);
    unsigned* X = a.ctl + 64 + x * xr::kXWords;
    unsigned* fault = a.ctl + xr::kFault;
    const long nframes = a.f.nframes;
    const unsigned ns = (unsigned)a.ns, C = (unsigned)a.chunk, lag = (unsigned)a.lag;

    // what ticket t waits on: its publication slot (or ~0u) and its counter (or null) + target
    auto deps = [&](unsigned t, unsigned& pslot, unsigned*& cnt, unsigned& target) {
        const unsigned s = t / TPS, q = t % TPS;
        pslot = ~0u;
        cnt = nullptr;
        target = 0;
        if (q < PPF) {
            pslot = q == 0 ? (s ? s - 1 : ~0u) : s;
            if (s >= ns) {
                cnt = xr::b_cnt(X, s % ns);
                target = PPF * (s / ns);
            }
        } else if (s >= lag) {
            pslot = s - lag;
            cnt = xr::a_cnt(X, pslot % ns);
            target = PPF * (pslot / ns + 1);
        }
    };
    auto prefetch = [&](unsigned t, XPre& pre) {
        unsigned pslot, target;
        unsigned* cnt;
        deps(t, pslot, cnt, target);
        pre.pub = pslot != ~0u ? __hip_atomic_load(xr::pub(X, pslot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        pre.cnt = cnt ? xr::ld_agent(cnt) : 0u;
    };
    auto pub_of = [&](unsigned slot, unsigned long long v) -> long {
        if ((unsigned)(v >> 32) == slot + 1) return (long)(v & 0xffffffffull);
        return xr::wait_pub(X, slot, fault);
    };
    auto wait_cnt = [&](unsigned* cnt, unsigned target, unsigned have) {
        if (a.nowait) return;  // TEMP ablation
        if (have < target) xr::spin_ge(cnt, target, fault);
    };
    // resolve ticket t: kind 0 skip, 1 A, 2 B, 3 exit
    auto resolve = [&](unsigned t, const XPre& pre, long& kind, long& fid, unsigned& slot) {
        const unsigned s = t / TPS, q = t % TPS;
        unsigned pslot, target;
        unsigned* cnt;
        deps(t, pslot, cnt, target);
        kind = 0;
        fid = 0;
        slot = s;
        if (q < PPF) {
            if (q == 0) {
                // claims are ordered per XCD (slot s claims after slot s - 1 published), so
                // a queue's frame ids only grow: once a slot is empty, all later ones are
                const long prev = s ? pub_of(s - 1, pre.pub) : -1;
                fid = (s % C == 0) ? (long)atomicAdd(a.ctl, C) : prev + 1;
                xr::publish(X, s, fid);
            } else {
                fid = pub_of(s, pre.pub);
            }
            if (fid < nframes) {
                if (cnt) wait_cnt(cnt, target, pre.cnt);
                kind = 1;
            }
        } else if (s >= lag) {
            slot = s - lag;
            fid = pub_of(slot, pre.pub);
            if (fid < nframes) {
                wait_cnt(cnt, target, pre.cnt);
                kind = 2;
            } else {
                kind = 3;
            }
        }
    };

    unsigned t1 = 0, t2 = 0;
    XPre pre{0ull, 0u};
    if (threadIdx.x == 0) {
        t1 = atomicAdd(X, 1u);
        t2 = atomicAdd(X, 1u);
        prefetch(t1, pre);
    }
    for (;;) {
        if (threadIdx.x == 0) {
            long kind, fid;
            unsigned slot;
            const unsigned tw = t1;
            resolve(tw, pre, kind, fid, slot);
            if (kind == 3) {
                // the drawn tickets not worked: a slot's first A ticket among them is published
                // empty (as every slot after an empty one) so no holder of that slot's other
                // tickets, and no next claimer, is left waiting for it
                if (t2 % TPS == 0) xr::publish(X, t2 / TPS, xr::kEmpty);
            } else {
                t1 = t2;
                t2 = atomicAdd(X, 1u);  // in flight during the piece
                prefetch(t1, pre);      // likewise: consumed at the end of the piece
            }
            desc[0] = kind | ((long)(tw % TPS % PPF) << 2) | ((long)slot << 8);
            desc[1] = fid;
        }
        __syncthreads();
        const long d = desc[0], fid = desc[1];
        const int kind = (int)(d & 3);
        const unsigned slot = (unsigned)(d >> 8);
        if (kind == 3) break;
        const int blk = (int)((d >> 2) & 63);
        if (kind == 1) {
            float2* S = a.ring + ((long)x * ns + slot % ns) * 65536L;
            f64_piece_a<CB>(a.f, fid, blk, lds, S, a.inpol);
            if (!a.nodrain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's scratch stores are in L2
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_fetch_add(xr::a_cnt(X, slot % ns), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (kind == 2) {
            const float2* S = a.ring + ((long)x * ns + slot % ns) * 65536L;
            f64_piece_b<CB>(a.f, fid, blk, lds, S, [&] {
                if (threadIdx.x == 0)
                    __hip_atomic_fetch_add(xr::b_cnt(X, slot % ns), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }, a.outpol);
            __syncthreads();  // LDS reuse by the next piece
        } else {
            __syncthreads();
        }
    }
}


// ---- launch excerpt (fft_launch, before the two-launch 64K path) ----
#if 0
    static const char* xenv = getenv("SDRGPU_F64X");  // TEMP: tuning
    if (p->M == 65536 && (!xenv || atoi(xenv) > 0)) {
        const int ns = xenv ? std::max(2, std::min(xr::kNsMax, atoi(xenv))) : 4;
        static const char* cenv = getenv("SDRGPU_F64X_C");
        const int chunk = cenv ? std::max(1, atoi(cenv)) : 8;
        static const char* wenv = getenv("SDRGPU_F64X_W");
        const int wpc = wenv ? std::max(1, atoi(wenv)) : 2;
        static const char* benv = getenv("SDRGPU_F64X_CB");
        const int cbx = benv ? atoi(benv) : 32;
        static const char* lenv = getenv("SDRGPU_F64X_L");
        const int lag = std::max(1, std::min(ns - 1, lenv ? atoi(lenv) : 2));
        if (scratch_frames * (size_t)p->M * sizeof(float2) <
            xr::kCtlBytes + (size_t)xr::kXcd * ns * p->M * sizeof(float2))
            return SDRGPU_ERR_UNSUPPORTED;
        static int ncu = [] {
            int dev = 0, n = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
                n = 256;
            return n;
        }();
        F64XArgs a{};
        a.f.src = src;
        a.f.nframes = fr.nframes;
        a.f.tw = p->tw4096;
        a.f.twM = p->twM;
        a.f.norm = p->norm;
        a.f.store_mode = store_mode;
        a.f.out = out;
        a.ctl = reinterpret_cast<unsigned*>(scratch);
        a.ring = reinterpret_cast<float2*>(reinterpret_cast<char*>(scratch) + xr::kCtlBytes);
        a.ns = ns;
        a.chunk = chunk;
        a.lag = lag;
        static const char* nwenv = getenv("SDRGPU_F64X_NOWAIT");
        a.nowait = nwenv ? atoi(nwenv) : 0;
        static const char* ipenv = getenv("SDRGPU_F64X_IN");
        static const char* openv = getenv("SDRGPU_F64X_OUT");
        a.inpol = ipenv ? atoi(ipenv) : 0;
        a.outpol = openv ? atoi(openv) : 0;
        static const char* ndenv = getenv("SDRGPU_F64X_NODRAIN");
        a.nodrain = ndenv ? atoi(ndenv) : 0;
        SDRGPU_HIP_TRY(hipMemsetAsync(a.ctl, 0, xr::kCtlWords * sizeof(unsigned), s));
        const long pieces = 2 * fr.nframes * (256 / cbx);
        const long grid = std::min<long>((long)wpc * ncu, std::max<long>(8, pieces));
        if (cbx == 16)
            hipLaunchKernelGGL(fft64k_xcd_kernel<16>, dim3((unsigned)grid), dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL(fft64k_xcd_kernel<32>, dim3((unsigned)grid), dim3(512), 0, s, a);
        SDRGPU_LAUNCH_CHECK();
        return SDRGPU_OK;
    }
#endif
