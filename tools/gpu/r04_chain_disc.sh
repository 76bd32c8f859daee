#!/bin/bash
# Round 4: configs[3] chain mismatch with the ONE FIR build -- does it need the PLL's LDS?
# The LDS-free pll_kernel ("scalar": lock flags at an odd address) against the split kernel,
# with the ONE library (fir_ablate.sh one) and with the product library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_chain_disc}
mkdir -p $O
cd $R
MAKEFLAGS=-j16 VARIANTS="one" timeout -k 10 600 bash tools/experiments/fir_ablate.sh > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
i=0
for cut in ${CUTS:-3000}; do
for lib in ${LIBS:-one prod one prod}; do
  for m in ${MODES:-scalar split}; do
    i=$((i + 1))
    f=$O/${i}_${lib}_${m}_$cut.txt
    if [ $lib = prod ]; then
      timeout -k 10 180 python -u tools/diag/c4_snap_diag.py $cut 0 $m > $f 2>&1 || { tail -20 $f; exit 2; }
    else
      timeout -k 10 180 python -u tools/experiments/run_with_lib.py tools/experiments/abl/lib_$lib.so tools/diag/c4_snap_diag.py $cut 0 $m > $f 2>&1 || { tail -20 $f; exit 2; }
    fi
    echo "== $lib $m cut $cut"; grep -h "PLL\|^  " $f
  done
done
done
