#!/bin/bash
# Build PLL instruction-selection variants of libsdrgpu into tools/experiments/abl/lib_<v>.so
#   noslp: pll.hip without SLP vectorisation (no packed-f32 pairs in the libm chains)
#   opq:   atanf's common-path value made opaque before the final selects (no exec branch)
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v "/pll.o")
for v in ${VARIANTS:-noslp opq noslp_opq}; do
  d=tools/pllv_$v
  rm -rf $d && mkdir -p $d && cp unnamed-rust-sdr_amd/csrc/*.h unnamed-rust-sdr_amd/csrc/*.hpp unnamed-rust-sdr_amd/csrc/pll.hip $d/
  FLAGS=""
  case $v in *noslp*) FLAGS="-fno-slp-vectorize";; esac
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
