#!/bin/bash
# Round-2 GPU check: GPU tests, smoke, default bench, kernel-trace stats of the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_check}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest died rc=$rc"; tail -30 $O/pytest_gpu.log; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 2; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 3; }
tail -1 $O/bench.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 4; }
echo done
