#!/bin/bash
# Build copies of the headline FIR kernel with one constant changed into
# tools/experiments/abl/lib_<v>.so (never into the product library), plus libbase.so = the
# product build.  VARIANTS="run2 run4 run16" (kRunTiles), u8runN (kRunTilesU8),
# d1runN (D = 1 banks dealt in blocked runs of N tiles), wg4 (two 4-wave
# workgroups per CU).  Run one with:
#   python tools/experiments/run_with_lib.py tools/experiments/abl/lib_<v>.so bench.py ...
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/experiments/abl
make -C unnamed-rust-sdr_amd -s
cp unnamed-rust-sdr_amd/libsdrgpu.so tools/experiments/abl/libbase.so
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v fir_mxh.o)
for v in ${VARIANTS:-run2 run4 run16}; do
  src=tools/experiments/abl/fir_mxh_$v.hip
  cp unnamed-rust-sdr_amd/csrc/fir_mxh.hip $src
  case $v in
    gsrun*) n=${v#gsrun}; sed -i "s/^constexpr int kRunTiles = [0-9]*;/constexpr int kRunTiles = $n;/; s/^constexpr int kRunTilesU8 = [0-9]*;/constexpr int kRunTilesU8 = $n;/; s/^    p.blocked = run > 0;/    p.blocked = 0;/" $src
          grep -q "kRunTiles = $n;" $src && grep -q "p.blocked = 0;" $src ;;
    run*) n=${v#run}; sed -i "s/^constexpr int kRunTiles = [0-9]*;/constexpr int kRunTiles = $n;/" $src
          grep -q "kRunTiles = $n;" $src ;;
    u8run*) n=${v#u8run}; sed -i "s/^constexpr int kRunTilesU8 = [0-9]*;/constexpr int kRunTilesU8 = $n;/" $src
          grep -q "kRunTilesU8 = $n;" $src ;;
    d1run*) n=${v#d1run}; sed -i "s/(u8 ? kRunTilesU8 : kRunTiles) : 0;/(u8 ? kRunTilesU8 : kRunTiles) : $n;/" $src
          grep -q "kRunTiles) : $n;" $src ;;
    wg4) # two 4-wave workgroups per CU (finer end-time granularity), 2 x CUs workgroups
          sed -i "s/^constexpr int kWaves = 8; .*/constexpr int kWaves = 4;/; s/std::min((long)cus, ceil_div(p.units, kWaves))/std::min(2L * cus, ceil_div(p.units, kWaves))/" $src
          grep -q "kWaves = 4;" $src && grep -q "2L \* cus" $src ;;
    xcd) # XCD-aware range map: the 8 XCDs (dispatch slot b % 8) each stream one contiguous eighth
          python3 - $src <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
a = "    const long wave = (long)blockIdx.x * kWaves + wv;"
assert a in s
s = s.replace(a, a + "\n    const long bxr = gridDim.x % 8 == 0 ? (long)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : (long)blockIdx.x;")
for o, n in (("((long)blockIdx.x + 1) * p.units / gridDim.x", "(bxr + 1) * p.units / gridDim.x"),
             ("(long)blockIdx.x * p.units / gridDim.x + wv", "bxr * p.units / gridDim.x + wv")):
    assert o in s
    s = s.replace(o, n)
open(p, 'w').write(s)
PY
          ;;
    gstride) # runs dealt grid-strided (all CUs stream one chip-wide window) instead of per-WG ranges
          sed -i "s/^    p.blocked = run > 0;/    p.blocked = 0;/" $src
          grep -q "p.blocked = 0;" $src ;;
    noprio) sed -i "s/^    if (wv >= kWaves \/ 2) __builtin_amdgcn_s_setprio(1);//" $src
          ! grep -q "s_setprio(1);" $src ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
    -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip -c $src -o tools/experiments/abl/fir_mxh_$v.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/lib_$v.so \
    tools/experiments/abl/fir_mxh_$v.o $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built lib_$v.so"
done
