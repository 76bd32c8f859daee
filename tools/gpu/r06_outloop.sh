#!/bin/bash
# Round 6: exact tiles after the main loop (fir_mxh.hip) -- the inf / NaN and FIR tests, bitwise
# outputs on finite data against the in-loop build, then alternating A/Bs against the session's
# starting library and the in-loop build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_outloop}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_fir_gpu.py tests/test_firbank_gpu.py tests/test_in_place_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_inloop.so tools/diag/fir_bitwise.py $O/a.npz > $O/bitwise.txt 2>&1 &&
timeout -k 10 200 python -u tools/diag/fir_bitwise.py $O/b.npz >> $O/bitwise.txt 2>&1 &&
python tools/diag/fir_bitwise.py --compare $O/a.npz $O/b.npz >> $O/bitwise.txt 2>&1
rc=$?; rm -f $O/a.npz $O/b.npz; grep -E "identical|differ" $O/bitwise.txt; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python -u tools/diag/nonfinite_rate.py > $O/rate.txt 2>&1 && head -2 $O/rate.txt
OUT=${OUT:-r06_outloop}/ab REPS=${REPS:-4} KINDS=${KINDS:-"c64 bank"} ARMS="start=tools/diag/var_build/lib_start.so inloop=tools/diag/var_build/lib_inloop.so new=product" bash tools/gpu/ab.sh
