#!/bin/bash
# Resampler parity on the GPU (sdrgpu_src_* vs the libsamplerate restatement).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/src
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_resample.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
