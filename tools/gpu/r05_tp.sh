#!/bin/bash
# Round 5: the time-parallel PLL -- PLL / chain / signal GPU tests, then bench_configs c4.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_tp}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_pll_gpu.py tests/test_firbank_gpu.py tests/test_fm_chain_gpu.py tests/test_signal.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench_configs.py --config c4 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 2; }
cut -c1-900 $O/c4.jsonl
