#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -q -p no:cacheprovider -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
case "$(tail -1 gpurun_out/pytest_gpu.log)" in *"rc=0"|*"rc=1") ;; *) echo "pytest died"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo os > gpurun_out/bench_os.log 2>&1 || exit 2
timeout -k 10 300 python -m pytest tests/test_fir_gpu.py -m gpu -q -p no:cacheprovider -k "full_size" > gpurun_out/pytest_full.log 2>&1
echo "rc=$?" >> gpurun_out/pytest_full.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_os -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --algo os > $R/gpurun_out/prof.log 2>&1 || exit 3
echo done
