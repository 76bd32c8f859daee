#!/bin/bash
# u8 FIR: ingest + FIR GPU tests, then the c2u8 line (3 reps).
set -o pipefail
O=gpurun_out/u8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ingest_gpu.py tests/test_fir_gpu.py tests/test_rtltcp.py tests/test_stream_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench_configs.py --config c2u8 --no-cpu-baseline > $O/c2u8_$rep.jsonl 2> $O/c2u8.err || { tail -20 $O/c2u8.err; exit 2; }
  python3 -c "
import json
for l in open('$O/c2u8_$rep.jsonl'):
    if l.startswith('{'): d=json.loads(l); print('rep $rep', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
