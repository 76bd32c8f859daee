#!/bin/bash
# A/B of experiment libraries (tools/experiments/abl/lib_*.so) against the product library
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # $1 = variant (base = product), rest = script args
  local v=$1; shift
  if [ $v = base ]; then timeout -k 10 200 python "$@"; else timeout -k 10 200 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so "$@"; fi
}
FIRV=${FIRV:-}
PLLV=${PLLV:-base}
for rep in 1 2; do
  for v in $FIRV; do
    run $v bench.py --no-cpu-baseline --steps 30 > gpurun_out/var_$v.log 2>gpurun_out/var_$v.err || { tail -5 gpurun_out/var_$v.err; exit 1; }
    echo "fir $v $(tail -1 gpurun_out/var_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"])')"
  done
  for v in $PLLV; do
    run $v bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 17 > gpurun_out/var_$v.log 2>gpurun_out/var_$v.err || { tail -5 gpurun_out/var_$v.err; exit 2; }
    echo "pll $v $(tail -1 gpurun_out/var_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["pll_ns_per_sample_chain"])')"
  done
done
