#!/bin/bash
# Round 5 chain discriminator libraries (tools/diag/probe_build/lib_<bank>_<pll>.so): the ONE
# or the product FIR bank with the PLL's split / LDS-free kernel capped in VGPRs
# (tools/diag/pll_vgpr_variant.py).  Diagnostic only; never the product library.
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
O=tools/diag/probe_build
mkdir -p $O
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip"
bash tools/experiments/one_source.sh $O/fir_mxh_one.hip
/opt/rocm/bin/hipcc $F -c $O/fir_mxh_one.hip -o $O/fir_one.o &
cp unnamed-rust-sdr_amd/build/fir_mxh.o $O/fir_prod.o
# name split_cap scalar_cap route
VARS="orig:0:0:split:- scalar96:0:5:scalar:- split80:6:0:split:- scalar80:0:6:scalar:- splitx:0:0:split:excl scalarx:0:0:scalar:excl"
for v in $VARS; do
  IFS=: read name sc kc route ex <<< "$v"
  python3 tools/diag/pll_vgpr_variant.py $O/pll_$name.hip $sc $kc $route $ex
  /opt/rocm/bin/hipcc $F -ffp-contract=off -c $O/pll_$name.hip -o $O/pll_$name.o &
done
wait
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v -e '/fir_mxh.o' -e '/pll.o')
for bank in one prod; do
  for v in $VARS; do
    name=${v%%:*}
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/lib_${bank}_$name.so $OBJS $O/fir_$bank.o $O/pll_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  done
done
ls $O/*.so
