#!/bin/bash
# Exhaustive atanf reduction-division check, then the PLL tests + c4 lines.
set -o pipefail
O=gpurun_out/pllsplit
mkdir -p $O
timeout -k 10 120 ./tools/atanf_check > $O/atanf_check.log 2>&1 || { cat $O/atanf_check.log; exit 4; }
cat $O/atanf_check.log
bash tools/gpu/r02_pllsplit.sh
