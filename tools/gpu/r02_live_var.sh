#!/bin/bash
# 1000-point live-spectrum block/tile variants (tools/experiments/abl/lib_live*.so), 2 reps.
set -o pipefail
O=gpurun_out/livev
mkdir -p $O
for r in 1 2; do
for v in default 128_2048 256_4096 256_2048; do
  if [ $v = default ]; then cmd="python bench_configs.py"; else cmd="python tools/experiments/run_with_lib.py tools/experiments/abl/lib_live$v.so bench_configs.py"; fi
  timeout -k 10 200 $cmd --config ex --no-cpu-baseline > $O/ex_$v.jsonl 2> $O/ex_$v.err || { tail -5 $O/ex_$v.err; exit 2; }
  python3 -c "
import json
for l in open('$O/ex_$v.jsonl'):
    if 'ex_live' in l: d=json.loads(l); print('$v rep $r', d['roofline']['kernel_ms'], d['value'])"
done
done
