#!/bin/bash
# dB store fast path: FFT GPU tests (incl. dB parity) + the examples' FFT shapes.
set -o pipefail
O=gpurun_out/db
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fft_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench_configs.py --config ex --no-cpu-baseline > $O/ex.jsonl 2> $O/ex.err || { tail -20 $O/ex.err; exit 2; }
python3 -c "
import json
for l in open('$O/ex.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['config'][:40], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
