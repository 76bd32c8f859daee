#!/bin/bash
# rtl_tcp u8 ingest: parity tests (fused + converted shapes), regression on the FIR tests,
# then the c2u8 bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/u8
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ingest_gpu.py tests/test_fir_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench_configs.py --config c2u8 > $O/c2u8.log 2>&1 || { tail -5 $O/c2u8.log; exit 2; }
tail -1 $O/c2u8.log
