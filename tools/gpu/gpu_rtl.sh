#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rtl
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_rtltcp.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
