#!/bin/bash
# Sinc resampler: GPU parity (bit-exact vs the oracle) + bench lines.
set -o pipefail
O=gpurun_out/sinc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resample.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench_configs.py --config src --no-cpu-baseline > $O/src.jsonl 2> $O/src.err || { tail -20 $O/src.err; exit 2; }
cut -c1-400 $O/src.jsonl
