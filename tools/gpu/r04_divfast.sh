#!/bin/bash
# Round 4: the headline kernel without the per-unit 64-bit division for one stream: FIR +
# bank/PLL chain tests, then the driver-window / steady-state A/B against the round-3 library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_divfast}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fir_gpu.py tests/test_firbank_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
OUT=${OUT:-r04_divfast}/ab NOBUILD=1 VARIANTS=base KINDS="c64" REPS=${REPS:-4} bash tools/gpu/r04_var.sh
