#!/bin/bash
# Build the configs[3] chain probe libraries (tools/diag/probe_build/lib_hw_<name>.so): the
# product objects with fir_mxh.o replaced by an instrumented bank (start-only HW_ID records) and
# pll.o by an instrumented PLL (tools/diag/pll_probe_patch.py).  Diagnostic only.
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
O=tools/diag/probe_build
mkdir -p $O
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip"
python3 tools/diag/pll_vgpr_variant.py $O/pll_scalar96.hip 0 5 scalar
bash tools/experiments/one_source.sh $O/fir_mxh_one.hip
# name bank_src pll_src opts
VARS="one_split:$O/fir_mxh_one.hip:unnamed-rust-sdr_amd/csrc/pll.hip:-
one_shadow:$O/fir_mxh_one.hip:unnamed-rust-sdr_amd/csrc/pll.hip:--shadow
one_scalar96:$O/fir_mxh_one.hip:$O/pll_scalar96.hip:-
prod_split:unnamed-rust-sdr_amd/csrc/fir_mxh.hip:unnamed-rust-sdr_amd/csrc/pll.hip:-"
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v -e '/fir_mxh.o' -e '/pll.o')
for v in $VARS; do
  IFS=: read name bsrc psrc opt <<< "$v"
  python3 tools/diag/pll_probe_patch.py $O/hw_pll_$name.hip $bsrc $O/hw_fir_$name.hip --pll-src=$psrc $opt
  ( /opt/rocm/bin/hipcc $F -ffp-contract=off -c $O/hw_pll_$name.hip -o $O/hw_pll_$name.o -Rpass-analysis=kernel-resource-usage 2> $O/hw_pll_$name.res &&
    /opt/rocm/bin/hipcc $F -c $O/hw_fir_$name.hip -o $O/hw_fir_$name.o -Rpass-analysis=kernel-resource-usage 2> $O/hw_fir_$name.res &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/lib_hw_$name.so $OBJS $O/hw_pll_$name.o $O/hw_fir_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib ) &
done
wait
for v in $VARS; do
  name=${v%%:*}
  echo "$name: bank D=1 NCH=9 $(grep -A2 'ILi9ELb0ELi1ELi3E' $O/hw_fir_$name.res | grep -m1 -o 'VGPRs: [0-9]*')," \
       "pll main.rs split $(grep -A2 'pll_split_kernelILb0ELi0ELi1ELi0ELi0E' $O/hw_pll_$name.res | grep -m1 -o 'VGPRs: [0-9]*')," \
       "scalar $(grep -A2 'pll_kernelILb0ELi0ELi1ELi0ELi0ELb1E' $O/hw_pll_$name.res | grep -m1 -o 'VGPRs: [0-9]*')"
done
