#!/bin/bash
# Round 6: inf / NaN samples through fir_mxh (exact_tile) -- the new tests on the product and on
# the previous build (tools/diag/var_build/lib_prev.so), bitwise outputs on finite data against
# the previous build, then alternating per-launch A/Bs (configs[1], configs[4] bank).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_nf}
mkdir -p $O
cd $R
T="tests/test_fir_gpu.py -k nonfinite"
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests_new.txt 2>&1 || { tail -30 $O/tests_new.txt; exit 1; }
tail -1 $O/tests_new.txt
timeout -k 10 200 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_prev.so -m pytest -q --timeout 120 --timeout-method thread -m gpu $T > $O/tests_prev.txt 2>&1
tail -1 $O/tests_prev.txt
timeout -k 10 120 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_prev.so tools/diag/fir_bitwise.py $O/prev.npz > $O/bitwise.txt 2>&1 &&
timeout -k 10 120 python -u tools/diag/fir_bitwise.py $O/prod.npz >> $O/bitwise.txt 2>&1 &&
python tools/diag/fir_bitwise.py --compare $O/prev.npz $O/prod.npz >> $O/bitwise.txt 2>&1
rc=$?
rm -f $O/prev.npz $O/prod.npz
tail -6 $O/bitwise.txt
[ $rc -le 1 ] || exit 3
OUT=${OUT:-r06_nf}/ab REPS=${REPS:-3} KINDS=${KINDS:-"c64 bank"} ARMS="prev=tools/diag/var_build/lib_prev.so new=product" bash tools/gpu/ab.sh
