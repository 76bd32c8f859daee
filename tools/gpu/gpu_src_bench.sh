#!/bin/bash
# Resampler: parity tests, bench line, rocprof kernel trace of the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/srcb
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_resample.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config src --steps 20 --warmup 3 > $O/src.log 2>&1 || { tail -20 $O/src.log; exit 2; }
tail -1 $O/src.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench_configs.py --config src --steps 20 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
find $O/prof -name "*kernel_stats.csv" | head -3
