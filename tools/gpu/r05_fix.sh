#!/bin/bash
# Round 5: the PLL co-residency fix.  (1) the new concurrent PLL-beside-bank test against the
# pre-fix PLL (tools/diag/probe_build/lib_pre_r5_pll.so: expected to FAIL) and the product
# library; (2) the driver's GPU suite; (3) PLL ns per sample-chain (bench_configs c4).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_fix}
mkdir -p $O
cd $R
T="tests/test_firbank_gpu.py::test_pll_beside_concurrent_mfma_bank"
timeout -k 10 300 python -u tools/experiments/run_with_lib.py tools/diag/probe_build/lib_pre_r5_pll.so -m pytest -x -q -p no:cacheprovider "$T" > $O/pre_fix.log 2>&1; echo "pre-fix PLL: rc $?"; tail -3 $O/pre_fix.log
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider "$T" > $O/fix.log 2>&1 || { tail -30 $O/fix.log; exit 1; }
tail -1 $O/fix.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 2; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u bench_configs.py --config c4 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 3; }
cut -c1-600 $O/c4.jsonl
# (4) the hazard in isolation (tools/diag/pk_mfma_probe.hip, prebuilt): victim alone / beside MFMA waves / owning its SIMD
for m in 0 1 2; do
  timeout -k 10 120 tools/diag/probe_build/pk_mfma_probe $m 2000000 1600000 >> $O/pk_mfma_probe.txt 2>&1 || { tail -5 $O/pk_mfma_probe.txt; exit 4; }
done
cat $O/pk_mfma_probe.txt
