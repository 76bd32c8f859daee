#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bq
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_biquad_gpu.py tests/test_pll_gpu.py tests/test_signal.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
