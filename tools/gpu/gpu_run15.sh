#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/test_fir_gpu.py tests/test_fft_gpu.py tests/test_signal.py -m gpu -x -q > gpurun_out/pytest_pk.log 2>&1 || { tail -40 gpurun_out/pytest_pk.log; exit 2; }
tail -2 gpurun_out/pytest_pk.log
rm -f gpurun_out/variants.txt
for v in 1 1; do
SDRGPU_OS_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --algo os > gpurun_out/bench_v$v.log 2>&1 || exit 3
python -c "
import json; d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/variants.txt
done
timeout -k 10 300 python bench_configs.py --config c3 --no-cpu-baseline > gpurun_out/c3.log 2>&1 || exit 4
cat gpurun_out/variants.txt; tail -1 gpurun_out/c3.log
