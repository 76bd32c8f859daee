#!/bin/bash
# GPU test pass: pytest -m gpu [extra pytest args], log under gpurun_out/$OUT/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_tests}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider "$@" > $O/pytest.log 2>&1
rc=$?
tail -30 $O/pytest.log
exit $rc
