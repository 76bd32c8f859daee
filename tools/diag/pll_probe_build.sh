#!/bin/bash
# Build the configs[3] chain probe library (tools/diag/probe_build/lib_probe.so): the product
# objects with fir_mxh.o replaced by the instrumented ONE build and pll.o by the instrumented
# PLL (tools/diag/pll_probe_patch.py).  Diagnostic only; never the product library.
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
O=tools/diag/probe_build
mkdir -p $O
python3 tools/diag/pll_probe_patch.py $O/pll_probe.hip ${BANK_SRC:-tools/experiments/fir_mxh_one.hip} $O/fir_mxh_probe.hip
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip"
/opt/rocm/bin/hipcc $F -ffp-contract=off -c $O/pll_probe.hip -o $O/pll_probe.o &
/opt/rocm/bin/hipcc $F -c $O/fir_mxh_probe.hip -o $O/fir_mxh_probe.o &
wait
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v -e '/fir_mxh.o' -e '/pll.o')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/lib_probe.so $OBJS $O/pll_probe.o $O/fir_mxh_probe.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $O/lib_probe.so
