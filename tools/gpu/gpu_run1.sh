#!/bin/bash
# GPU pass: parity tests, short bench, rocprof kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
case "$(tail -1 gpurun_out/pytest_gpu.log)" in *"rc=0"|*"rc=1") ;; *) echo "pytest died"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --log2n 24 > gpurun_out/bench24.log 2>&1 || exit 2
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1 || exit 3
echo done
