#!/bin/bash
# Build variants of the int8-MFMA u8 FIR kernel (fir_mxi.hip) into tools/experiments/abl/
# (never into the product library).  Run one with:
#   python tools/experiments/run_with_lib.py tools/experiments/abl/lib_mxi_<v>.so tools/gpu/series.py --kind u8
#   gs2 / gs4 : units of 2 / 4 tiles dealt grid-strided (the c64 headline's dealing)
#   b4 / b16  : per-workgroup runs of 4 / 16 tiles (product: 8)
#   w16       : two 8-wave workgroups per CU (4 waves per SIMD, <= 128 VGPRs)
#   cs2 / cs4 : tiles of 2 / 4 column sets (2 / 4 KiB of raw samples in flight per wave)
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/experiments/abl
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v fir_mxi.o)
for v in ${VARIANTS:-gs2}; do
  src=tools/experiments/abl/fir_mxi_$v.hip
  cp unnamed-rust-sdr_amd/csrc/fir_mxi.hip $src
  python3 - $src $v <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]; s = open(p).read()
def rep(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new)
if v.startswith("gs"):
    rep("constexpr int kRunTiles = 8;", "constexpr int kRunTiles = %s;" % v[2:])
    rep("const long ub1 = ((long)blockIdx.x + 1) * p.units / gridDim.x;", "const long ub1 = p.units;")
    rep("if (++c.t >= c.nt) seek(c, c.u + kWaves);", "if (++c.t >= c.nt) seek(c, c.u + (long)gridDim.x * kWaves);")
    rep("seek(cm, (long)blockIdx.x * p.units / gridDim.x + wv);", "seek(cm, (long)blockIdx.x * kWaves + wv);")
elif v.startswith("b"):
    rep("constexpr int kRunTiles = 8;", "constexpr int kRunTiles = %s;" % v[1:])
elif v.startswith("cs"):  # cs2 / cs4: 2 / 4 column sets (2 / 4 x 1024 new samples) per staged window
    rep("constexpr int kCs = 1;", "constexpr int kCs = %s;" % v[2:])
elif v == "w16":
    rep("__attribute__((amdgpu_waves_per_eu(2, 2)))", "__attribute__((amdgpu_waves_per_eu(4, 4)))")
    rep("std::min((long)cus, ceil_div(p.units, kWaves))", "std::min(2L * cus, ceil_div(p.units, kWaves))")
else:
    raise SystemExit("unknown variant " + v)
open(p, 'w').write(s)
PY
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip -c $src -o tools/experiments/abl/fir_mxi_$v.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/lib_mxi_$v.so $OBJS tools/experiments/abl/fir_mxi_$v.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
echo built
