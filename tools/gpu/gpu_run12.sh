#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -x -q > gpurun_out/pytest_d2.log 2>&1 || { tail -30 gpurun_out/pytest_d2.log; exit 2; }
tail -3 gpurun_out/pytest_d2.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo direct > gpurun_out/bench_d2.log 2>&1 || exit 3
tail -1 gpurun_out/bench_d2.log
SDRGPU_DIRECT_V1=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo direct > gpurun_out/bench_d1.log 2>&1 || exit 4
tail -1 gpurun_out/bench_d1.log
