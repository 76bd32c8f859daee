#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
case "$(tail -1 gpurun_out/pytest_gpu.log)" in *"rc=0"|*"rc=1") ;; *) echo "pytest died"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo os > gpurun_out/bench_os2.log 2>&1 || exit 2
SDRGPU_OS_V1=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo os > gpurun_out/bench_os1.log 2>&1 || exit 2
echo done
