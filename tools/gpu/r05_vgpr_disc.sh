#!/bin/bash
# Round 5: configs[3] chain discriminator over PLL VGPR caps (tools/diag/pll_vgpr_build.sh,
# prebuilt here): which (bank build, PLL kernel, PLL VGPRs) pairs mismatch the oracle?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_vgpr_disc}
mkdir -p $O
cd $R
for v in ${VARS:-one_orig one_scalar96 one_split80 prod_split80 prod_scalar80 prod_orig}; do
  f=$O/$v.txt
  timeout -k 10 180 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_$v.so tools/diag/c4_snap_diag.py ${CUT:-3000} 0 split > $f 2>&1 || { tail -20 $f; exit 2; }
  echo "== $v"; grep -h "PLL\|^  " $f
done
