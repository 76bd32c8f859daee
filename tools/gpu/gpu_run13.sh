#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/dvariants.txt
timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -x -q > gpurun_out/pytest_d4.log 2>&1 || { tail -30 gpurun_out/pytest_d4.log; exit 2; }
tail -2 gpurun_out/pytest_d4.log
for v in 4 3 2 4; do
SDRGPU_DIRECT_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --algo direct > gpurun_out/bench_dv$v.log 2>&1 || exit 3
python -c "
import json; d=json.loads(open('gpurun_out/bench_dv$v.log').read().strip().splitlines()[-1]); print('dvariant $v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/dvariants.txt
done
SDRGPU_DIRECT_VARIANT=3 timeout -k 10 600 python -m pytest tests/test_fir_gpu.py -m gpu -x -q -k "direct" > gpurun_out/pytest_d3.log 2>&1 || { tail -30 gpurun_out/pytest_d3.log; exit 4; }
tail -1 gpurun_out/pytest_d3.log
cat gpurun_out/dvariants.txt
