#!/bin/bash
# Round 5: one instrumented run of the configs[3] chain reproducer (ONE bank build beside the
# split PLL), tools/diag/c4_probe_diag.py on tools/diag/probe_build/lib_probe.so (prebuilt here).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_probe}
mkdir -p $O
cd $R
for cut in ${CUTS:-3000}; do
  timeout -k 10 240 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_probe.so tools/diag/c4_probe_diag.py $cut > $O/probe_$cut.txt 2>&1 || { tail -30 $O/probe_$cut.txt; exit 2; }
  head -40 $O/probe_$cut.txt
done
