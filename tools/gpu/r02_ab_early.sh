#!/bin/bash
# A/B: product FIR vs fir_ablate.sh 'early' (tile k+1 staged and tile k+2's loads issued before
# tile k's MFMAs instead of interleaved with them); bench.py --steps 30, alternating.
set -o pipefail
O=gpurun_out/abearly
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > $O/base$rep.json 2>/dev/null || exit 1
  line="rep $rep base $(python3 -c "import json; print(json.load(open('$O/base$rep.json'))['roofline']['kernel_ms'])")"
  for v in ${VARIANTS:-early}; do
    timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so bench.py --no-cpu-baseline --steps 30 > $O/$v$rep.json 2>/dev/null || exit 2
    line="$line | $v $(python3 -c "import json; print(json.load(open('$O/$v$rep.json'))['roofline']['kernel_ms'])")"
  done
  echo "$line"
done
