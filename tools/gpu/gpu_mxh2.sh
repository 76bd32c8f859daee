#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mxh2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fir_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "mx" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --algo mx --no-cpu-baseline --steps 20 > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 3; }
  python -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
for nt in 0 1 2 3; do run nt$nt SDRGPU_MXH_NT=$nt; done
for S in 64 16; do run seg$S SDRGPU_MXL_SEG=$S; run seg${S}_nt3 SDRGPU_MXL_SEG=$S SDRGPU_MXH_NT=3; done
