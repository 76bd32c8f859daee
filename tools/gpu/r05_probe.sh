#!/bin/bash
# Round 5: the configs[3] chain reproducer with placement records (tools/diag/pll_probe_build.sh,
# prebuilt here): does each (bank build, PLL build) pair co-reside on CUs, and is it wrong?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_probe}
mkdir -p $O
cd $R
for v in ${VARS:-one_shadow one_split one_scalar96 prod_split}; do
  f=$O/probe_$v.txt
  PROBE_NPZ=$O/probe_$v.npz timeout -k 10 240 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_hw_$v.so tools/diag/c4_probe_diag.py ${CUT:-3000} > $f 2>&1 || { tail -30 $f; exit 2; }
  echo "== $v"; grep -h "SUMMARY\|hand-off\|mismatch classes\|wave 0 chain" $f | cut -c1-300
done
