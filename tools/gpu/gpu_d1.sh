#!/bin/bash
# fp16 MFMA FIR at D=1 (FIR banks, configs[3] matched filter and configs[4]): full GPU tests,
# then c5 / c4 bench lines (new default vs overlap-save).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/d1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config c5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 2; }
tail -1 $O/c5.log | cut -c1-330
SDRGPU_MX_VARIANT=1 timeout -k 10 300 python bench_configs.py --config c5 --no-cpu-baseline > $O/c5_os.log 2>&1 || { tail -5 $O/c5_os.log; exit 3; }
tail -1 $O/c5_os.log | cut -c1-330
