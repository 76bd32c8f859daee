#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mxl2
mkdir -p $O
cd $R
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --algo mx --no-cpu-baseline --steps 20 > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 3; }
  python -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
for S in 256 64 16 4; do
run full_S$S SDRGPU_MX_ABLATION=0 SDRGPU_MXL_SEG=$S
run mem_S$S SDRGPU_MX_ABLATION=1 SDRGPU_MXL_SEG=$S
done
