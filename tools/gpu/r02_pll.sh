#!/bin/bash
# fast-division check on the GPU, PLL parity, c4 timing
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./tools/fdiv_check > gpurun_out/fdiv.log 2>&1 || { tail -8 gpurun_out/fdiv.log; exit 1; }
tail -2 gpurun_out/fdiv.log
timeout -k 10 300 python -u -m pytest tests/test_pll_gpu.py tests/test_firbank_gpu.py tests/test_stream_gpu.py tests/test_signal.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pll_pytest.log 2>&1 || { tail -30 gpurun_out/pll_pytest.log; exit 2; }
tail -1 gpurun_out/pll_pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 18 > gpurun_out/c4_$r.log 2>&1 || exit 3
  tail -1 gpurun_out/c4_$r.log | cut -c1-330
done
