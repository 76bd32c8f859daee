#!/bin/bash
# Round 6: the new GPU tests (in-place biquad / PLL, the PLL's adapted plan on noise, the
# concurrent-bank PLL at the time-parallel size) on the product library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_new}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_pll_gpu.py::test_pll_in_place_long_block tests/test_pll_gpu.py::test_pll_time_parallel_adapts_to_misses \
  tests/test_biquad_gpu.py::test_biquad_in_place_long_block "tests/test_firbank_gpu.py::test_pll_beside_concurrent_mfma_bank" \
  > $O/new_tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $O/new_tests.txt | head -40
exit $rc
