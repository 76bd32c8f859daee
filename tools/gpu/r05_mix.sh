#!/bin/bash
# Round 5: the fma_mix staging build against the shipped one -- bitwise outputs
# (tools/diag/fir_bitwise.py), the FIR GPU tests, then the per-launch A/B (tools/gpu/ab.sh).
set -o pipefail
O=gpurun_out/${OUT:-r05_mix}
mkdir -p $O
BASE=${BASE:-tools/diag/probe_build/lib_cur.so}
timeout -k 10 120 python -u tools/experiments/run_with_lib.py $BASE tools/diag/fir_bitwise.py $O/base.npz > $O/bitwise.txt 2>&1 &&
timeout -k 10 120 python -u tools/diag/fir_bitwise.py $O/new.npz >> $O/bitwise.txt 2>&1 &&
python tools/diag/fir_bitwise.py --compare $O/base.npz $O/new.npz >> $O/bitwise.txt 2>&1
rc=$?
rm -f $O/base.npz $O/new.npz
[ $rc -le 1 ] || exit 3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fir_gpu.py tests/test_firbank_gpu.py > $O/fir_tests.txt 2>&1 || exit 4
OUT=${OUT:-r05_mix} REPS=${REPS:-3} KINDS=${KINDS:-c64} ARMS=${ARMS:-"cur=$BASE new=product"} bash tools/gpu/ab.sh > $O/ab.txt 2>&1
