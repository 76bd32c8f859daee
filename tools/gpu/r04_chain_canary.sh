#!/bin/bash
# Round 4: configs[3] chain with the ONE FIR build -- does the split PLL's mismatch need a
# bank workgroup on the same CU, and does the bank write LDS outside its allocation?
# canary = D = 1 launches take 16 KiB more LDS (no PLL workgroup fits beside them) holding a
# pattern that is checked at the end (printf CANARY on any change).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_chain_canary}
mkdir -p $O
cd $R
MAKEFLAGS=-j16 VARIANTS="one+canary canary one" timeout -k 10 600 bash tools/experiments/fir_ablate.sh > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
i=0
for lib in one+canary canary one+canary one; do
  i=$((i + 1))
  f=$O/${i}_${lib}_split.txt
  timeout -k 10 180 python -u tools/experiments/run_with_lib.py tools/experiments/abl/lib_$lib.so tools/diag/c4_snap_diag.py 3000 0 split > $f 2>&1 || { tail -20 $f; exit 2; }
  echo "== $lib split: CANARY lines $(grep -c CANARY $f || true)"; grep -h "PLL" $f
done
