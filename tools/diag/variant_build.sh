#!/bin/bash
# Build a variant of libsdrgpu.so with extra compile flags on ONE source file:
#   bash tools/diag/variant_build.sh NAME SOURCE.hip "FLAGS"  ->  tools/diag/var_build/lib_NAME.so (git-ignored; travels with the snapshot)
# (e.g. fir_mxh.hip "-DSDRGPU_MXR=1" with tools/experiments/fir_mxh_rolesplit.patch applied).  The product library is
# rebuilt first; the variant links every other product object unchanged.  Diagnostic only.
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
O=tools/diag/var_build
mkdir -p $O
src=$2
obj=$(basename ${src%.hip}).o
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $3 \
  -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip -c unnamed-rust-sdr_amd/csrc/$src -o $O/var_$1.o
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v "/$obj")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/lib_$1.so $OBJS $O/var_$1.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f $O/var_$1.o
echo "built $O/lib_$1.so"
