#!/bin/bash
# Round 4: the int8-MFMA u8 kernel (fir_mxi.hip): u8 parity tests, then the driver-window /
# steady-state A/B against the round-3 library (tools/experiments/ab/lib_base.so = HEAD before it).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_mxi}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ingest_gpu.py tests/test_rtltcp.py tests/test_fm_chain_gpu.py tests/test_stream_gpu.py \
  tests/test_random_sweep_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
OUT=${OUT:-r04_mxi}/ab VARIANTS=base KINDS=u8 REPS=${REPS:-3} bash tools/gpu/r04_var.sh
