#!/bin/bash
# MFMA FIR path: parity tests, then bench (full kernel + memory-only / compute-only ablations).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mx
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fir_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "${TK:-mx or auto}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for a in ${ABLS:-0 1 2}; do
SDRGPU_MX_ABLATION=$a timeout -k 10 300 python bench.py --algo mx --no-cpu-baseline --steps 20 > $O/bench_abl$a.log 2>&1 || { tail -5 $O/bench_abl$a.log; exit 3; }
python -c "
import json; d=json.loads(open('$O/bench_abl$a.log').read().strip().splitlines()[-1]); print('abl $a', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
