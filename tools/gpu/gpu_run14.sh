#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/variants.txt
SDRGPU_OS_VARIANT=9 timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -x -q -k "os or auto" > gpurun_out/pytest_v9.log 2>&1 || { tail -40 gpurun_out/pytest_v9.log; exit 2; }
tail -2 gpurun_out/pytest_v9.log
for v in 9 1 9; do
SDRGPU_OS_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo os > gpurun_out/bench_v$v.log 2>&1 || exit 3
python -c "
import json; d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/variants.txt
done
cat gpurun_out/variants.txt
