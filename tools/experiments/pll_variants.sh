#!/bin/bash
# Build PLL instruction-selection variants of libsdrgpu into tools/experiments/abl/lib_<v>.so
#   noslp: pll.hip without SLP vectorisation (no packed-f32 pairs in the libm chains)
#   opq:   atanf's common-path value made opaque before the final selects (no exec branch)
#   noballot: atan2f's special-case selects always evaluated (no uniform branch)
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v "/pll.o")
for v in ${VARIANTS:-noslp opq noslp_opq}; do
  d=tools/pllv_$v
  rm -rf $d && mkdir -p $d && cp unnamed-rust-sdr_amd/csrc/*.h unnamed-rust-sdr_amd/csrc/*.hpp unnamed-rust-sdr_amd/csrc/pll.hip $d/
  FLAGS=""
  case $v in *noslp*) FLAGS="-fno-slp-vectorize";; esac
  case $v in *noballot*)
    python3 - $d/libm_glibc.h <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    if (!__builtin_amdgcn_ballot_w64(spec)) return r;"
assert old in s
s = s.replace(old, "    (void)spec;")
open(p, 'w').write(s)
PY
  ;; esac
  case $v in abl_noatan|abl_nosincos|abl_nooff)  # timing-only ablations (results invalid)
    python3 - $d/pll.hip $v <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]; s = open(p).read()
if v == "abl_noatan":
    old = "sdr_atan2f_bfx(li, lr) * p.gain"; new = "(li * lr) * p.gain"
elif v == "abl_nosincos":
    old = "sdr_sincosf_bf2(phase, &sn, &cs);"; new = "sn = phase * 0.5f; cs = phase * 0.25f;"
else:
    a = s.index("        // off the loop-carried chain: lock / output filters and the output select")
    b = s.index("    };\n\n    // full chunks of kChunk samples")
    s = s[:a] + "        ov = phasedif; lv = 0;\n" + s[b:]
    old = new = ""
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
PY
  ;; esac
  case $v in *opq*)
    python3 - $d/libm_glibc.h <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "    return ix >= 0x4c000000 ? rhuge : ix < 0x31000000 ? x : small ? rsmall : rbig;"
assert old in s
s = s.replace(old, """    float rc = small ? rsmall : rbig;
#if defined(__HIP_DEVICE_COMPILE__)
    __asm__ volatile("" : "+v"(rc));
#endif
    return ix >= 0x4c000000 ? rhuge : ix < 0x31000000 ? x : rc;""")
open(p, 'w').write(s)
PY
  ;; esac
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off $FLAGS -I$d -Iinclude -x hip -c $d/pll.hip -o $d/pll.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/lib_$v.so $OBJS $d/pll.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
echo built
