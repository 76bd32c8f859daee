#!/bin/bash
# Round 6: which packed-f32 form fails beside the partner MFMA wave?  fir_mxh's
# batched exact sums built as explicit packed pairs (tools/experiments/fir_mxh_pkdiag.patch,
# tools/diag/variant_build.sh): pkd1 default operand selection + s_nop 0, pkd2 src0's low half
# in both lanes (op_sel_hi [0,1]) with no wait state (the compiler's failing form), pkd3 the
# same with s_nop 4.  tools/diag/nf_mismatch.py, 9 cases x 5 repetitions each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_pkdiag}
mkdir -p $O
cd $R
export REPS=5
for v in ${VARS:-pkd1 pkd2 pkd3}; do
  timeout -k 10 300 python -u tools/experiments/run_with_lib.py tools/diag/var_build/lib_$v.so tools/diag/nf_mismatch.py > $O/$v.txt 2>&1 || { tail $O/$v.txt; exit 1; }
  echo "== $v"; grep -E "^case" $O/$v.txt | awk '{s += $7; if ($7 > 0) b++} END {print NR " runs, " b+0 " with wrong outputs, " s+0 " wrong outputs"}'
done
