#!/bin/bash
# Round 6: the exact-sum fallbacks with batched loads -- inf / NaN tests, bitwise outputs on
# finite data against the previous build (tools/diag/var_build/lib_head.so), the NaN-heavy
# launch times (tools/diag/nonfinite_rate.py) of both builds, then per-launch A/Bs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_nfrate}
mkdir -p $O
cd $R
L=tools/diag/var_build/lib_head.so
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_fir_gpu.py -k "nonfinite or silent" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for t in fir_bitwise fir_paths_dump; do
  timeout -k 10 200 python -u tools/experiments/run_with_lib.py $L tools/diag/$t.py $O/a.npz > $O/bitwise_$t.txt 2>&1 &&
  timeout -k 10 200 python -u tools/diag/$t.py $O/b.npz >> $O/bitwise_$t.txt 2>&1 &&
  python tools/diag/fir_bitwise.py --compare $O/a.npz $O/b.npz >> $O/bitwise_$t.txt 2>&1
  rc=$?; rm -f $O/a.npz $O/b.npz
  grep -c identical $O/bitwise_$t.txt; grep differ $O/bitwise_$t.txt
  [ $rc -le 1 ] || exit 3
done
timeout -k 10 300 python -u tools/experiments/run_with_lib.py $L tools/diag/nonfinite_rate.py > $O/rate_head.txt 2>&1 || { tail $O/rate_head.txt; exit 4; }
timeout -k 10 300 python -u tools/diag/nonfinite_rate.py > $O/rate_new.txt 2>&1 || { tail $O/rate_new.txt; exit 5; }
cat $O/rate_head.txt $O/rate_new.txt
OUT=${OUT:-r06_nfrate}/ab REPS=${REPS:-3} KINDS=${KINDS:-"c64 bank"} ARMS="head=$L new=product" bash tools/gpu/ab.sh
