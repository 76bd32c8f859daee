#!/bin/bash
# Round 4: rtl_tcp u8 FIR without decimation on the int8 kernel: u8 parity tests, the u8
# parity spot check, then the A/B against the library before it (lib_base: converts the
# block to c64 and runs the fp16 D = 1 kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_u8d1}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ingest_gpu.py tests/test_rtltcp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/diag/u8_parity.py > $O/parity.txt 2>&1 || { tail -20 $O/parity.txt; exit 2; }
cat $O/parity.txt
OUT=${OUT:-r04_u8d1}/ab NOBUILD=1 VARIANTS=base KINDS="u8d1 u8 bank" REPS=${REPS:-2} bash tools/gpu/r04_var.sh
