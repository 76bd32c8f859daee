#!/bin/bash
# Build fft_gen.hip with compile-time overrides into tools/experiments/abl/libfgv_<name>.so:
# fft_gen_variant.sh NAME "-DLIVE_BLK=256 -DLIVE_TILE=5120"
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/experiments/abl
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v fft_gen.o)
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude $2 -x hip -c unnamed-rust-sdr_amd/csrc/fft_gen.hip -o tools/experiments/abl/fft_gen_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/libfgv_$1.so $OBJS tools/experiments/abl/fft_gen_$1.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $1
