#!/bin/bash
# FIR dynamic tail pools: FIR GPU tests (incl. the whole-stream and full-size checks), then
# the headline bench against the previous build (tools/experiments/abl/lib_prepool.so).
set -o pipefail
O=gpurun_out/pool
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fir_gpu.py tests/test_ingest_gpu.py tests/test_firbank_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > $O/new$rep.json 2>/dev/null || exit 2
  timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_prepool.so bench.py --no-cpu-baseline --steps 30 > $O/old$rep.json 2>/dev/null || exit 3
  python3 -c "
import json; a=json.load(open('$O/new$rep.json')); b=json.load(open('$O/old$rep.json'))
print('rep $rep pool', a['roofline']['kernel_ms'], a['roofline']['frac'], '| prev', b['roofline']['kernel_ms'], b['roofline']['frac'])"
done
