#!/bin/bash
# Build ablated copies of the headline FIR kernel into tools/experiments/abl/ (never into the
# product library): nomfma = MFMAs replaced by one VALU add per fragment (LDS reads kept),
# noload = every fast-path tile load reads the 8 KiB dummy buffer (compute + stores only).
# Run one with: python tools/experiments/run_with_lib.py tools/experiments/abl/lib_<v>.so bench.py ...
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/experiments/abl
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v fir_mxh.o)
for v in ${VARIANTS:-nomfma noload}; do
  src=tools/experiments/abl/fir_mxh_$v.hip  # (v may be composite, e.g. clk+nomfma)
  cp unnamed-rust-sdr_amd/csrc/fir_mxh.hip $src
  for part in ${v//+/ }; do  # composite variants: a+b applies a, then b
  if [ $part = nomfma ]; then
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);"""
assert old in s
s = s.replace(old, """    c[0] += __uint_as_float(b[0] & 0x3ffu);
    return c;""")
open(p, 'w').write(s)
PY
  elif [ $part = noload ]; then
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "const float2* src2 = fast2 ? p.in + ld.ch * p.ld_in + j2 : p.dummy;"
assert old in s
s = s.replace(old, "const float2* src2 = p.dummy;")
old = """            const unsigned* src2u = fast2 ? p.in_u8 + ld.ch * (p.ld_in / 2) + (j2 >> 1)
                                          : reinterpret_cast<const unsigned*>(p.dummy);"""
assert old in s  # the rtl_tcp u8 launch's tile loads too
s = s.replace(old, "            const unsigned* src2u = reinterpret_cast<const unsigned*>(p.dummy);")
open(p, 'w').write(s)
PY
  elif [ $part = prio ]; then  # static s_setprio 1 for the younger half (waves 4-7) of the workgroup
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);"
assert old in s
s = s.replace(old, old + "\n    if (wv >= kWaves / 2) __builtin_amdgcn_s_setprio(1);")
open(p, 'w').write(s)
PY
  elif [ $part = stplain ]; then  # plain (temporal) output stores instead of non-temporal
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """                    __builtin_nontemporal_store(y0, o4);
                    __builtin_nontemporal_store(y1, o4 + 1);"""
assert old in s
s = s.replace(old, """                    o4[0] = y0;
                    o4[1] = y1;""")
open(p, 'w').write(s)
PY
  elif [ $part = ldplain ]; then  # plain loads for the streamed tiles instead of non-temporal
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """                        const f32x4 r = __builtin_nontemporal_load(
                            reinterpret_cast<const f32x4*>(src2 + 128 * k + 2 * lane));"""
assert old in s
s = s.replace(old, """                        const f32x4 r = *reinterpret_cast<const f32x4*>(src2 + 128 * k + 2 * lane);""")
open(p, 'w').write(s)
PY
  elif [ $part = wvdiv ]; then  # wave index left divergent (VGPR cursor math, no SGPR spills)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);"
assert old in s
s = s.replace(old, "const int wv = threadIdx.x >> 6;")
open(p, 'w').write(s)
PY
  elif [ $part = nohist ]; then  # history groups not re-staged per window (wrong outputs: cost probe)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "                    for (int k = 0; k < NH; ++k) put(WN + hist_addr(k), hr[k], scn);"
assert old in s
s = s.replace(old, "                    for (int k = 0; k < NH; ++k) if (scn == 0.f) put(WN + hist_addr(k), hr[k], scn);")
open(p, 'w').write(s)
PY
  elif [ $part = nosplit ]; then  # hi plane only, lo = 0 (wrong precision: split-VALU cost probe)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    lo = pk_rtz(a - lo_f(hi), b - hi_f(hi));"
assert old in s
s = s.replace(old, "    lo = 0u;")
open(p, 'w').write(s)
PY
  elif [ $part = nomax ]; then  # fixed window scale (no abs-max / wave reduction: cost probe)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "            return wave_scale(m);"
assert old in s
s = s.replace(old, "            return 15;")
open(p, 'w').write(s)
PY
  elif [ $part = early ]; then  # stage all of tile k+1 and issue all of tile k+2's loads BEFORE tile k's MFMAs
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old_a = """            read_frags(fb[0], 0, 0);
#pragma unroll
            for (int i = 0; i < CS * NCH; ++i) {"""
new_a = """#pragma unroll
            for (int k = 0; k < NH; ++k) put(WN + hist_addr(k), hr[k], scn);
            if (ld_run) load_hist(hr, ld);
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                put(WN + new_addr(k), nx[k], scn);
                if (k >= NG - NH) keep[k - (NG > NH ? NG - NH : 0)] = nx[k];
                if constexpr (U8) {
                    nx[k] = __builtin_nontemporal_load(src2u + 64 * k + lane);
                } else {
                    const f32x4 r = __builtin_nontemporal_load(
                        reinterpret_cast<const f32x4*>(src2 + 128 * k + 2 * lane));
                    nx[k] = make_float4(r[0], r[1], r[2], r[3]);
                }
            }
            read_frags(fb[0], 0, 0);
#pragma unroll
            for (int i = 0; i < CS * NCH; ++i) {"""
assert old_a in s
s = s.replace(old_a, new_a)
old_b = """                if (i == 0) {  // window k+1's history (old hr); then tile k+2's, if it opens a run"""
i0 = s.index(old_b)
i1 = s.index("            }\n            if (!ld_run) {", i0)
s = s[:i0] + s[i1:]
open(p, 'w').write(s)
PY
  elif [ $part = mfma4 ]; then  # the two taps-hi x samples-lo MFMAs dropped (4 of 6 per chunk; wrong precision: MFMA-count probe)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """                    if (!U8) {
                        cr[j] = mfma(ah[c], f[1], cr[j]);
                        ci[j] = mfma(ah[c], f[3], ci[j]);
                    }"""
assert old in s
s = s.replace(old, "")
open(p, 'w').write(s)
PY
  elif [ $part = wgtime ]; then  # per-workgroup start/end s_memrealtime (100 MHz) into out[0..511]: tail census
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    const int lane = threadIdx.x & 63;"
assert old in s
s = s.replace(old, "    const unsigned long long t_wg0 = __builtin_amdgcn_s_memrealtime();\n" + old, 1)
old2 = "    if (p.hist_next) {  // stream history carry, spread over the whole grid"
assert old2 in s
s = s.replace(old2, """    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        unsigned long long* o = reinterpret_cast<unsigned long long*>(p.out) + 2 * blockIdx.x;
        o[0] = t_wg0 | ((unsigned long long)(xcc & 7) << 56);
        o[1] = t_end;
    }
""" + old2, 1)
open(p, 'w').write(s)
PY
  elif [ $part = clk ]; then  # per-workgroup shader-clock / 100 MHz ticks over the launch, 16 B per workgroup at out - 4 KiB (timing-only: the caller reserves that space)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    const int lane = threadIdx.x & 63;"
assert old in s
s = s.replace(old, "    const unsigned long long c_wg0 = __builtin_readcyclecounter();\n"
                   "    const unsigned long long t_wg0 = __builtin_amdgcn_s_memrealtime();\n" + old, 1)
old2 = "    if (p.hist_next) {  // stream history carry, spread over the whole grid"
assert old2 in s
s = s.replace(old2, """    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long c_end = __builtin_readcyclecounter();
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        unsigned long long* o = reinterpret_cast<unsigned long long*>(p.out) - 512 + 2 * (blockIdx.x & 255);
        o[0] = t_end - t_wg0;
        o[1] = c_end - c_wg0;
    }
""" + old2, 1)
open(p, 'w').write(s)
PY
  elif [ $part = mprio ]; then  # priority 1 while a wave issues each chunk's MFMAs, 0 for its staging (no static per-wave priority)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    if (wv >= kWaves / 2) __builtin_amdgcn_s_setprio(1);"
assert old in s
s = s.replace(old, "")
old = """                    __builtin_amdgcn_sched_barrier(0);
                    const u32x4(&f)[4] = fb["""
assert old in s
s = s.replace(old, """                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_s_setprio(1);
                    const u32x4(&f)[4] = fb[""")
old = """                    cr[j] = mfma(ah[c], f[0], cr[j]);
                    ci[j] = mfma(ah[c], f[2], ci[j]);
                }"""
assert old in s
s = s.replace(old, """                    cr[j] = mfma(ah[c], f[0], cr[j]);
                    ci[j] = mfma(ah[c], f[2], ci[j]);
                    __builtin_amdgcn_sched_barrier(0);
                    __builtin_amdgcn_s_setprio(0);
                }""")
open(p, 'w').write(s)
PY
  elif [ $part = frag2 ]; then  # B fragments read two chunks ahead (three slots) when no fragment is shared (D = 4)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "            u32x4 fb[2][4];"
assert old in s
s = s.replace(old, "            u32x4 fb[3][4];")
old = """            read_frags(fb[0], 0, 0);
            // D = 1"""
assert old in s
s = s.replace(old, """            read_frags(fb[0], 0, 0);
            if (D == 4 && CS * NCH > 1) read_frags(fb[1], 1, 0);
            // D = 1""")
old = """                    const int ni = i + 1;
                    const bool reuse = kShare && ni % NCH == 0;
                    if (ni < CS * NCH && !reuse)
                        read_frags(fb[(kShare ? ni - ni / NCH : ni) & 1], ni % NCH, ni / NCH);
                    __builtin_amdgcn_sched_barrier(0);
                    const u32x4(&f)[4] = fb[(kShare ? i - j : i) & 1];"""
assert old in s
s = s.replace(old, """                    const int ni = i + (D == 4 ? 2 : 1);
                    const bool reuse = kShare && ni % NCH == 0;
                    if (ni < CS * NCH && !reuse)
                        read_frags(fb[D == 4 ? ni % 3 : (kShare ? ni - ni / NCH : ni) & 1], ni % NCH, ni / NCH);
                    __builtin_amdgcn_sched_barrier(0);
                    const u32x4(&f)[4] = fb[D == 4 ? i % 3 : (kShare ? i - j : i) & 1];""")
open(p, 'w').write(s)
PY
  elif [ $part = stag ]; then  # staggered MFMA / staging phases for the ONE launch (tools/experiments/fir_mxh_staggered.patch; round 4: slower, not kept)
    patch -s $src tools/experiments/fir_mxh_staggered.patch
  elif [ $part = noone ]; then  # the ONE instantiation compiled but never launched (bisect)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    const bool one = !u8 && D == 4"
assert old in s
s = s.replace(old, "    const bool one = false && !u8 && D == 4")
open(p, 'w').write(s)
PY
  elif [ $part = r3src ]; then  # the round-3 fir_mxh.hip (commit 76500ef), rebuilt (bisect)
    git show 76500ef:unnamed-rust-sdr_amd/csrc/fir_mxh.hip > $src
  elif [ $part = one ]; then  # round 4's ONE instantiation + factored body (tools/experiments/one_source.sh): faster, but the configs[3] chain test mismatched beside it until the PLL waves owned their SIMD
    bash tools/experiments/one_source.sh $src
  elif [ $part = canary ]; then  # D = 1 launches get 16 KiB more LDS (a CU then holds no other workgroup beside a bank workgroup), filled with a pattern and checked at the end (printf CANARY on a change)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    extern __shared__ __attribute__((aligned(16))) char smem[];"
assert old in s
s = s.replace(old, old + """
    unsigned* canary = reinterpret_cast<unsigned*>(smem + kWaves * G::WAVE);
    if constexpr (D == 1) {
        for (int q = threadIdx.x; q < 4096; q += kBlock) canary[q] = 0xA5A5A5A5u ^ (unsigned)q;
        __syncthreads();
    }""")
old = "    if (p.hist_next) {  // stream history carry, spread over the whole grid"
assert old in s
s = s.replace(old, """    if constexpr (D == 1) {
        __syncthreads();
        int bad = -1;
        unsigned val = 0;
        for (int q = threadIdx.x; q < 4096; q += kBlock)
            if (canary[q] != (0xA5A5A5A5u ^ (unsigned)q) && bad < 0) {
                bad = q;
                val = canary[q];
            }
        const unsigned long long m = __ballot(bad >= 0);
        if (m && (threadIdx.x & 63) == __ffsll((long long)m) - 1)
            printf("CANARY blk %d thr %d dword %d val %08x lanes %016llx\\n", (int)blockIdx.x, (int)threadIdx.x, bad, val, m);
    }
""" + old)
import re
n = len(re.findall(r"::WAVE\), s, p\)", s))
assert n == 1, n
s = re.sub(r"::WAVE\), s, p\)", "::WAVE) + (DD == 1 ? 16384 : 0), s, p)", s)
open(p, 'w').write(s)
PY
  elif [ $part = pkmul ]; then  # the window scale applied with v_pk_mul_f32 (two samples' components per instruction)
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """    unsigned h, l;
    split2(f.x * sc, f.z * sc, h, l);
    st32(lds, a, h);
    st32(lds, a + PLB, l);
    split2(f.y * sc, f.w * sc, h, l);"""
assert old in s
s = s.replace(old, """    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 s2 = {sc, sc};
    const f32x2 p0 = f32x2{f.x, f.y} * s2, p1 = f32x2{f.z, f.w} * s2;
    unsigned h, l;
    split2(p0[0], p1[0], h, l);
    st32(lds, a, h);
    st32(lds, a + PLB, l);
    split2(p0[1], p1[1], h, l);""")
open(p, 'w').write(s)
PY
  elif [ $part = wg2 ]; then  # two 4-wave workgroups per CU instead of one 8-wave workgroup
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
for old, new in (("constexpr int kWaves = 8;               // two waves per SIMD", "constexpr int kWaves = 4;  // x 2 workgroups per CU"),
                 ("const long W = (long)kWaves * cus;", "const long W = (long)kWaves * 2 * cus;"),
                 ("std::min((long)cus, ceil_div(p.units, kWaves))", "std::min(2L * cus, ceil_div(p.units, kWaves))")):
    assert old in s, old
    s = s.replace(old, new)
open(p, 'w').write(s)
PY
  elif [ $part = mfma16 ]; then  # each 16x16x32 MFMA as two 16x16x16 ones over the two K halves of the same fragments
    python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = """    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);"""
assert old in s
s = s.replace(old, """    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    const f16x8 a8 = __builtin_bit_cast(f16x8, a), b8 = __builtin_bit_cast(f16x8, b);
    const f16x4 alo = {a8[0], a8[1], a8[2], a8[3]}, ahi = {a8[4], a8[5], a8[6], a8[7]};
    const f16x4 blo = {b8[0], b8[1], b8[2], b8[3]}, bhi = {b8[4], b8[5], b8[6], b8[7]};
    c = __builtin_amdgcn_mfma_f32_16x16x16f16(alo, blo, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x16f16(ahi, bhi, c, 0, 0, 0);""")
open(p, 'w').write(s)
PY
  elif [ $part = lomask2 ] || [ $part = lomask3 ]; then  # low mantissa bits of the lo planes cleared (MFMA switching energy)
    python3 - $src $part <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]; s = open(p).read()
m = {'lomask2': '0xFFFCFFFCu', 'lomask3': '0xFFF8FFF8u'}[v]
old = "    lo = pk_rtz(a - lo_f(hi), b - hi_f(hi));"
assert old in s
s = s.replace(old, "    lo = pk_rtz(a - lo_f(hi), b - hi_f(hi)) & " + m + ";")
old2 = "                al[c][jj] = lw;"
assert old2 in s
s = s.replace(old2, "                al[c][jj] = lw & " + m + ";")
open(p, 'w').write(s)
PY
  elif [ $part = mfmaord ] || [ $part = dualacc ]; then  # MFMA operand order (switching energy)
    python3 - $src $part <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]; s = open(p).read()
old = """                    cr[j] = mfma(al[c], f[0], cr[j]);
                    ci[j] = mfma(al[c], f[2], ci[j]);
                    if (!U8) {
                        cr[j] = mfma(ah[c], f[1], cr[j]);
                        ci[j] = mfma(ah[c], f[3], ci[j]);
                    }
                    cr[j] = mfma(ah[c], f[0], cr[j]);
                    ci[j] = mfma(ah[c], f[2], ci[j]);"""
assert old in s
if v == 'mfmaord':  # A changes once per chunk (al, al, ah, ah, ah, ah)
    new = """                    cr[j] = mfma(al[c], f[0], cr[j]);
                    ci[j] = mfma(al[c], f[2], ci[j]);
                    cr[j] = mfma(ah[c], f[0], cr[j]);
                    ci[j] = mfma(ah[c], f[2], ci[j]);
                    if (!U8) {
                        cr[j] = mfma(ah[c], f[1], cr[j]);
                        ci[j] = mfma(ah[c], f[3], ci[j]);
                    }"""
else:  # second accumulator pair: consecutive MFMAs share their B operand
    new = """                    cr[j] = mfma(al[c], f[0], cr[j]);
                    cr2[j] = mfma(ah[c], f[0], cr2[j]);
                    ci[j] = mfma(al[c], f[2], ci[j]);
                    ci2[j] = mfma(ah[c], f[2], ci2[j]);
                    if (!U8) {
                        cr[j] = mfma(ah[c], f[1], cr[j]);
                        ci[j] = mfma(ah[c], f[3], ci[j]);
                    }"""
    o2 = """            f32x4 cr[CS], ci[CS];
#pragma unroll
            for (int j = 0; j < CS; ++j) {
                cr[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                ci[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }"""
    assert o2 in s
    s = s.replace(o2, o2.replace("f32x4 cr[CS], ci[CS];", "f32x4 cr[CS], ci[CS], cr2[CS], ci2[CS];").replace(
        "ci[j] = f32x4{0.f, 0.f, 0.f, 0.f};", "ci[j] = f32x4{0.f, 0.f, 0.f, 0.f};\n                cr2[j] = ci2[j] = cr[j];"))
    o3 = "            const int so = -(s_cur + p.sh);"
    assert o3 in s
    s = s.replace(o3, """#pragma unroll
            for (int j = 0; j < CS; ++j) {
                cr[j] += cr2[j];
                ci[j] += ci2[j];
            }
""" + o3)
s = s.replace(old, new)
open(p, 'w').write(s)
PY
  fi
  done
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip -c $src -o tools/experiments/abl/fir_mxh_$v.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/lib_$v.so $OBJS tools/experiments/abl/fir_mxh_$v.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
echo built
