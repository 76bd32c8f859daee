#!/bin/bash
# Round 6: the role-split headline kernel (fir_mxh.hip fir_mxr_kernel, built as
# tools/diag/var_build/lib_mxr.so by tools/diag/variant_build.sh) -- FIR GPU tests on it, then
# alternating per-launch A/Bs against the product (driver window = launches 6-25, steady state).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_mxr}
mkdir -p $O
cd $R
V=${V:-mxr}
timeout -k 10 400 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_$V.so -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_fir_gpu.py} > $O/fir_tests_$V.txt 2>&1 || { tail -30 $O/fir_tests_$V.txt; exit 4; }
tail -2 $O/fir_tests_$V.txt
OUT=${OUT:-r06_mxr}/ab REPS=${REPS:-3} KINDS=${KINDS:-c64} ARMS=${ARMS:-"new=product $V=tools/diag/var_build/lib_$V.so"} bash tools/gpu/ab.sh > $O/ab.txt 2>&1
cat $O/ab.txt
