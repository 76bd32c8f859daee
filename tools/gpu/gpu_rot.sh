#!/bin/bash
# fir_mxh per-unit start rotation (SDRGPU_MXH_ROT): parity, then A/B vs rot=0.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rot
mkdir -p $O
cd $R
true
true
for rep in 1 2 3 4; do
for r in 0 5 64; do
SDRGPU_MXH_ROT=$r timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > $O/b${r}_$rep.log 2>&1 || { tail -5 $O/b${r}_$rep.log; exit 2; }
echo "rot=$r rep=$rep $(tail -1 $O/b${r}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
done
