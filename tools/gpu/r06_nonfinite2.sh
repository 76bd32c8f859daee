#!/bin/bash
# Round 6: inf / NaN samples through the secondary FIR kernels (VALU direct forms, overlap-save,
# bf16x3 MFMA: fir_exact.hpp) -- the tests on the product and on the previous build
# (tools/diag/var_build/lib_prev.so), bitwise outputs on finite data, then per-launch A/Bs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_nf2}
mkdir -p $O
cd $R
T="tests/test_fir_gpu.py -k nonfinite"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu $T > $O/tests_new.txt 2>&1 || { tail -40 $O/tests_new.txt; exit 1; }
tail -1 $O/tests_new.txt
timeout -k 10 300 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_prev.so -m pytest -q --timeout 200 --timeout-method thread -m gpu $T > $O/tests_prev.txt 2>&1
grep -E "^FAILED|passed|failed" $O/tests_prev.txt | tail -12
timeout -k 10 200 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_prev.so tools/diag/fir_paths_dump.py $O/prev.npz > $O/bitwise.txt 2>&1 &&
timeout -k 10 200 python -u tools/diag/fir_paths_dump.py $O/prod.npz >> $O/bitwise.txt 2>&1 &&
python tools/diag/fir_bitwise.py --compare $O/prev.npz $O/prod.npz >> $O/bitwise.txt 2>&1
rc=$?
rm -f $O/prev.npz $O/prod.npz
tail -22 $O/bitwise.txt
[ $rc -le 1 ] || exit 3
OUT=${OUT:-r06_nf2}/ab REPS=${REPS:-2} KINDS=${KINDS:-"c64d8 c64dir4 c64dir1 c64os4 f32d1"} ARMS="prev=tools/diag/var_build/lib_prev.so new=product" bash tools/gpu/ab.sh
