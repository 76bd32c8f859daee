#!/bin/bash
# FFT GPU tests + the examples' FFT shapes (bench_configs ex): r02_fftq.sh <outdir>
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fftq}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_fft_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u bench_configs.py --config ex --no-cpu-baseline > $O/ex.jsonl 2> $O/ex.err || { tail -5 $O/ex.err; exit 2; }
python3 -c "
import json,sys
for l in open('$O/ex.jsonl'): d=json.loads(l); print(d['config'][:8], d['roofline']['kernel_ms'], d['roofline']['frac'])"
