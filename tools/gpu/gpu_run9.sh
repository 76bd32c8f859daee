#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
case "$(tail -1 gpurun_out/pytest_gpu.log)" in *"rc=0"|*"rc=1") ;; *) echo "pytest died"; exit 1;; esac
timeout -k 10 600 python bench_configs.py --config all --no-cpu-baseline > gpurun_out/bench_configs.log 2>&1 || exit 2
echo done
