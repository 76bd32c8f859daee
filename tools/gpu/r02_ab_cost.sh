#!/bin/bash
# Cost probes of the headline FIR's staging (fir_ablate.sh nohist / nosplit / nomax: results
# wrong by construction, timing only) against the product kernel; bench.py --steps 30.
set -o pipefail
O=gpurun_out/abcost
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > $O/base$rep.json 2>/dev/null || exit 1
  line="rep $rep base $(python3 -c "import json; print(json.load(open('$O/base$rep.json'))['roofline']['kernel_ms'])")"
  for v in nohist nosplit nomax; do
    timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so bench.py --no-cpu-baseline --steps 30 > $O/$v$rep.json 2>/dev/null || exit 2
    line="$line | $v $(python3 -c "import json; print(json.load(open('$O/$v$rep.json'))['roofline']['kernel_ms'])")"
  done
  echo "$line"
done
