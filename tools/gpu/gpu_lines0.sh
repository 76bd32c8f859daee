#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lines
mkdir -p $O
cd $R
SDRGPU_MXH_NT=7 timeout -k 10 400 python -u -m pytest tests/test_fir_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "K255D4n10000-mx" > $O/pytest7.log 2>&1 || { tail -8 $O/pytest7.log; exit 1; }
tail -1 $O/pytest7.log
