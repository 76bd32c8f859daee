#!/bin/bash
# PLL chain / helper-wave split: PLL GPU tests, then the c4 line (PLL-bound) 2 reps.
set -o pipefail
O=gpurun_out/pllsplit
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pll_gpu.py tests/test_biquad_gpu.py tests/test_signal.py tests/test_stream_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 18 > $O/c4_$r.log 2>&1 || { tail -5 $O/c4_$r.log; exit 3; }
  python3 -c "
import json
for l in open('$O/c4_$r.log'):
    if l.startswith('{'): d=json.loads(l); print('rep $r', {k: d[k] for k in d if k not in ('config', 'roofline', 'cpu_baseline')})"
done
