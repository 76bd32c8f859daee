#!/bin/bash
# Round 4: variants of the int8 u8 kernel (tools/experiments/mxi_ablate.sh, built here on the
# box): u8 parity spot check per variant, then the r04_var.sh A/B against the product library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_mxi_var}
mkdir -p $O
cd $R
MAKEFLAGS=-j16 VARIANTS="$MXI" timeout -k 10 600 bash tools/experiments/mxi_ablate.sh > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
timeout -k 10 300 python -u tools/diag/u8_parity.py > $O/parity_prod.txt 2>&1 || { tail -20 $O/parity_prod.txt; exit 2; }
tail -1 $O/parity_prod.txt
V=""
for v in $MXI; do
  timeout -k 10 300 python -u tools/experiments/run_with_lib.py tools/experiments/abl/lib_mxi_$v.so tools/diag/u8_parity.py > $O/parity_$v.txt 2>&1 || { tail -20 $O/parity_$v.txt; exit 2; }
  echo "$v: $(tail -1 $O/parity_$v.txt)"
  V="$V mxi_$v"
done
OUT=${OUT:-r04_mxi_var}/ab NOBUILD=1 VARIANTS="$V" KINDS=u8 REPS=${REPS:-3} bash tools/gpu/r04_var.sh
