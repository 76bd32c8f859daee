#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
SDRGPU_OS_VARIANT=${AV:-11} timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -x -q -k "os or auto" > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 2; }
tail -1 gpurun_out/pytest_ab.log
rm -f gpurun_out/variants.txt
for v in ${VLIST:-1 11 1 11}; do
SDRGPU_OS_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --algo os > gpurun_out/bench_v$v.log 2>&1 || exit 3
python -c "
import json; d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().splitlines()[-1]); print('variant $v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/variants.txt
done
cat gpurun_out/variants.txt
