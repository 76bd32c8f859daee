#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_pll_gpu.py tests/test_fir_gpu.py tests/test_fft_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
case "$(tail -1 gpurun_out/pytest_gpu.log)" in *"rc=0"|*"rc=1") ;; *) echo "pytest died"; exit 1;; esac
for v in 0 1 2; do
SDRGPU_OS_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo os > gpurun_out/bench_v$v.log 2>&1 || exit 2
done
SDRGPU_OS_VARIANT=1 SDRGPU_OS_VARIANT=1 timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 -k "os or auto" > gpurun_out/pytest_v1.log 2>&1; echo "rc=$?" >> gpurun_out/pytest_v1.log
echo done
