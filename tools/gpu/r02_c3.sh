#!/bin/bash
# FFT tests, c3 bench line, kernel trace of the c3 line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_c3}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fft_gpu.py tests/test_signal.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config c3 --no-cpu-baseline > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 2; }
tail -1 $O/c3.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench_configs.py --config c3 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 3; }
head -4 $O/trace/run_kernel_stats.csv
