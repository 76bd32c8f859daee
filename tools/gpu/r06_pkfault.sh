#!/bin/bash
# Round 6: the packed-f32 fault inside fir_mxh.  The inf / NaN tiles' exact sums
# (exact_tile) run in one wave while its SIMD partner issues MFMAs; tools/diag/nf_mismatch.py
# counts wrong finite outputs over 5 repetitions of 9 cases for: the product (exact sums as VOP2
# v_mul_f32 / v_add_f32), lib_pk (the same sums compiled to v_pk_mul_f32 -> v_pk_add_f32 pairs,
# 16 per batch) and lib_head (the committed one-at-a-time loop: one such pair per tap).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_pkfault}
mkdir -p $O
cd $R
export REPS=5
timeout -k 10 300 python -u tools/diag/nf_mismatch.py > $O/product.txt 2>&1 || { tail $O/product.txt; exit 1; }
timeout -k 10 300 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_pk.so tools/diag/nf_mismatch.py > $O/pk.txt 2>&1 || { tail $O/pk.txt; exit 2; }
timeout -k 10 300 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_head.so tools/diag/nf_mismatch.py > $O/head.txt 2>&1 || { tail $O/head.txt; exit 3; }
for f in product pk head; do echo "== $f"; grep -E "^case" $O/$f.txt | awk '{s += $7; if ($7 > 0) b++} END {print NR " runs, " b+0 " with wrong outputs, " s+0 " wrong outputs"}'; done
