#!/bin/bash
# Round 6: staged groups per MFMA chunk (fir_mxh.hip SDRGPU_SPC) -- bitwise outputs against the
# product (tools/diag/fir_bitwise.py: the staging order must not change a bit), the bank A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_spc2}
mkdir -p $O
cd $R
V=${V:-spc4}
timeout -k 10 120 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_$V.so tools/diag/fir_bitwise.py $O/var.npz > $O/bitwise.txt 2>&1 &&
timeout -k 10 120 python -u tools/diag/fir_bitwise.py $O/prod.npz >> $O/bitwise.txt 2>&1 &&
python tools/diag/fir_bitwise.py --compare $O/var.npz $O/prod.npz >> $O/bitwise.txt 2>&1
rc=$?
rm -f $O/var.npz $O/prod.npz
tail -8 $O/bitwise.txt
[ $rc -le 1 ] || exit 3
OUT=${OUT:-r06_spc2}/ab REPS=${REPS:-3} KINDS=${KINDS:-bank} ARMS="new=product $V=tools/diag/var_build/lib_$V.so" bash tools/gpu/ab.sh
