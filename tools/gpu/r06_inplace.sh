#!/bin/bash
# Round 6: in-place (overlapping) device calls on FIR / bank / FFT / STFT, then the FIR, bank,
# ingest and FFT suites again (run_dev gained the overlap check).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_inplace}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_in_place_gpu.py > $O/inplace.txt 2>&1 || { tail -40 $O/inplace.txt; exit 1; }
tail -3 $O/inplace.txt
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_fir_gpu.py tests/test_firbank_gpu.py tests/test_ingest_gpu.py tests/test_fft_gpu.py \
  > $O/suites.txt 2>&1; rc=$?
tail -5 $O/suites.txt
exit $rc
