#!/bin/bash
# Round 6: compile-time FFT kernels with the 32-bit-offset full-workgroup gather / store.
# FFT GPU tests on the product build, output hashes of base vs new (must be identical), then
# the live-spectrum timings of both builds alternated on the same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_fftfixed}
BASE=${BASE:-tools/diag/var_build/lib_base.so}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fft_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 2; }
tail -2 $O/tests.txt
timeout -k 10 120 python -u tools/experiments/run_with_lib.py $BASE tools/diag/fft_fixed_hash.py > $O/hash_base.txt 2>&1 || { tail -20 $O/hash_base.txt; exit 2; }
timeout -k 10 120 python -u tools/diag/fft_fixed_hash.py > $O/hash_new.txt 2>&1 || { tail -20 $O/hash_new.txt; exit 2; }
grep -v run_with_lib $O/hash_base.txt > $O/hash_base_only.txt
if diff $O/hash_base_only.txt $O/hash_new.txt > $O/hash_diff.txt; then echo "hashes identical ($(wc -l < $O/hash_new.txt) cases)"; else echo "HASHES DIFFER"; cat $O/hash_diff.txt; fi
# optional variant (VAR=path.so): its FFT tests, then a third timing arm
if [ -n "$VAR" ]; then
  timeout -k 10 300 python -u tools/experiments/run_with_lib.py $VAR -m pytest tests/test_fft_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_var.txt 2>&1 || { tail -30 $O/tests_var.txt; exit 2; }
  echo "variant: $(tail -1 $O/tests_var.txt)"
fi
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/experiments/run_with_lib.py $BASE tools/diag/stft_live_modes.py > $O/modes_base_$rep.txt 2>&1 || { tail -20 $O/modes_base_$rep.txt; exit 2; }
  timeout -k 10 120 python -u tools/diag/stft_live_modes.py > $O/modes_new_$rep.txt 2>&1 || { tail -20 $O/modes_new_$rep.txt; exit 2; }
  if [ -n "$VAR" ]; then
    timeout -k 10 120 python -u tools/experiments/run_with_lib.py $VAR tools/diag/stft_live_modes.py > $O/modes_var_$rep.txt 2>&1 || { tail -20 $O/modes_var_$rep.txt; exit 2; }
  fi
done
for f in $O/modes_*_*.txt; do echo "== $(basename $f)"; grep "^n=" $f; done
