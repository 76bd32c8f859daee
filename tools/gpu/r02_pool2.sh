#!/bin/bash
# pool build vs the same source with the pool disabled on the host vs the previous kernel
set -o pipefail
O=gpurun_out/pool2
mkdir -p $O
for rep in 1 2; do
  line="rep $rep"
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > $O/new$rep.json 2>/dev/null || exit 2
  line="$line pool $(python3 -c "import json; print(json.load(open('$O/new$rep.json'))['roofline']['kernel_ms'])")"
  for v in nopool prepool; do
    timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so bench.py --no-cpu-baseline --steps 30 > $O/$v$rep.json 2>/dev/null || exit 3
    line="$line | $v $(python3 -c "import json; print(json.load(open('$O/$v$rep.json'))['roofline']['kernel_ms'])")"
  done
  echo "$line"
done
