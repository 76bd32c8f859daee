#!/bin/bash
# Packed 14,400-point rfft: FFT GPU tests, then the examples' lines with kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rfft
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fft_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config ex --no-cpu-baseline > $O/ex.jsonl 2> $O/ex.err || { tail -20 $O/ex.err; exit 2; }
cut -c1-400 $O/ex.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench_configs.py --config ex --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -8
