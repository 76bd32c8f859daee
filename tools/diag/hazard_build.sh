#!/bin/bash
# Round 6 hazard reproducer libraries (tools/diag/probe_build/lib_haz_<arm>.so): round 4's ONE
# FIR bank (201 VGPRs: two bank waves leave a 96-VGPR PLL wave room on their SIMD) with the
# pre-fix PLL (own_simd() emptied), its device code taken through assembly and edited by
# tools/diag/pk_hazard_edit.py:
#   ctl       normal hipcc build of the pre-fix PLL
#   rt        device assembly -> assembler -> code object, unedited (checks the pipeline)
#   after12   s_nop 0 after every packed-f32 producer whose next instruction reads it as src1/2
#             and the compiler left without a wait state (op_sel_hi[0] = 0: the PLL mixer)
#   before12  the same number of s_nop 0 placed before those producers (timing control)
#   after0    s_nop 0 after the uncovered producers read as src0 only
#   all4      s_nop 4 after every packed-f32 instruction (the widest wait state)
#   oneclaim  the pre-fix PLL (ctl) beside the ONE bank built with the MFMA-side claim (v255)
# Diagnostic only; never the product library.  Needs the git history (one_source.sh).
set -e
cd "$(dirname "$0")/../.."
make -C unnamed-rust-sdr_amd -s
O=tools/diag/probe_build
L=/opt/rocm/lib/llvm/bin
mkdir -p $O
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip"
bash tools/experiments/one_source.sh $O/fir_mxh_one.hip
/opt/rocm/bin/hipcc $F -c $O/fir_mxh_one.hip -o $O/fir_one.o &
# oneclaim: the same ONE bank with the MFMA-side claim of common.hpp (each wave names v255)
python3 - $O/fir_mxh_one.hip $O/fir_mxh_oneclaim.hip <<'PY'
import sys
s = open(sys.argv[1]).read()
a = "    const int lane = threadIdx.x & 63;\n"
i = s.index("void fir_mxh_kernel(")
j = s.index(a, i)
open(sys.argv[2], "w").write(s[:j] + '    asm volatile("" ::: "v255");\n' + s[j:])
PY
/opt/rocm/bin/hipcc $F -c $O/fir_mxh_oneclaim.hip -o $O/fir_oneclaim.o &
sed 's/__device__ __forceinline__ void own_simd() { claim_simd_whole(); }/__device__ __forceinline__ void own_simd() {}/' \
  unnamed-rust-sdr_amd/csrc/pll.hip > $O/pll_nofix.hip
grep -q 'own_simd() {}' $O/pll_nofix.hip
/opt/rocm/bin/hipcc $F -ffp-contract=off -c $O/pll_nofix.hip -o $O/pll_ctl.o &
/opt/rocm/bin/hipcc $F -ffp-contract=off --cuda-device-only -S $O/pll_nofix.hip -o $O/pll_nofix.s &
wait
python3 tools/diag/pk_hazard_edit.py report $O/pll_nofix.s > $O/pll_nofix_census.txt
for arm in ${ARMS:-rt after12 before12 after0 all4}; do
  python3 tools/diag/pk_hazard_edit.py $arm $O/pll_nofix.s $O/pll_$arm.s
  $L/clang --target=amdgcn-amd-amdhsa -mcpu=gfx950 -c $O/pll_$arm.s -o $O/pll_${arm}_dev.o
  $L/ld.lld -shared $O/pll_${arm}_dev.o -o $O/pll_$arm.hsaco
  $L/clang-offload-bundler --type=o --targets=host-x86_64-unknown-linux-gnu-,hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=/dev/null --input=$O/pll_$arm.hsaco --output=$O/pll_$arm.fatbin
  $L/llvm-objcopy --update-section .hip_fatbin=$O/pll_$arm.fatbin $O/pll_ctl.o $O/pll_$arm.o
done
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v -e '/fir_mxh.o' -e '/pll.o')
for arm in ctl ${ARMS:-rt after12 before12 after0 all4}; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/lib_haz_$arm.so $OBJS $O/fir_one.o $O/pll_$arm.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/lib_haz_oneclaim.so $OBJS $O/fir_oneclaim.o $O/pll_ctl.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
# the round trip must reproduce the compiler's code object exactly
$L/llvm-objcopy --dump-section=.hip_fatbin=$O/ctl.fatbin $O/pll_ctl.o $O/junk.o
$L/clang-offload-bundler --unbundle --type=o --input=$O/ctl.fatbin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$O/pll_ctl.hsaco
for a in ctl rt; do $L/llvm-objdump -d --no-show-raw-insn $O/pll_$a.hsaco | sed 's/^ *[0-9a-f]*://' | tail -n +3 > $O/pll_$a.dis; done
cmp $O/pll_ctl.dis $O/pll_rt.dis && echo "round trip: identical instruction stream"
rm -f $O/junk.o $O/*.fatbin $O/*_dev.o $O/pll_*.dis $O/*.s $O/*.hsaco $O/*.o $O/*.hip
ls -la $O/lib_haz_*.so
