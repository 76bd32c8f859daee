#!/bin/bash
# A/B of fir_ablate.sh variants against the product headline kernel: r02_ab_fir.sh v1 v2 ...
mkdir -p gpurun_out/abfir
for rep in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/abfir/base$rep.json 2>/dev/null || exit 1
  line="rep $rep base $(python3 -c "import json; a=json.load(open('gpurun_out/abfir/base$rep.json')); print(a['roofline']['kernel_ms'])")"
  for v in "$@"; do
    timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so bench.py --no-cpu-baseline --steps 30 > gpurun_out/abfir/$v$rep.json 2>/dev/null || exit 1
    line="$line | $v $(python3 -c "import json; a=json.load(open('gpurun_out/abfir/$v$rep.json')); print(a['roofline']['kernel_ms'])")"
  done
  echo "$line"
done
