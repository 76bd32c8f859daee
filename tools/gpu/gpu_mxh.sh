#!/bin/bash
# fp16-split MFMA FIR (fir_mxh.hip): parity tests, then bench variants and ablations.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mxh
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fir_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "${TK:-mx or auto}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --algo mx --no-cpu-baseline --steps 20 > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; exit 3; }
  python -c "
import json; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
run mxh SDRGPU_MX_ABLATION=0
run mxh_mem SDRGPU_MX_ABLATION=1
run mxh_comp SDRGPU_MX_ABLATION=2
run mxl SDRGPU_MX_VARIANT=2
