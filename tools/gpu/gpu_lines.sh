#!/bin/bash
# Line-complete output stores (SDRGPU_MXH_NT=7) vs the default (3): parity, then A/B benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lines
mkdir -p $O
cd $R
SDRGPU_MXH_NT=7 timeout -k 10 400 python -u -m pytest tests/test_fir_gpu.py tests/test_ingest_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest7.log 2>&1 || { tail -40 $O/pytest7.log; exit 1; }
tail -1 $O/pytest7.log
for rep in 1 2 3; do
for nt in 3 7; do
SDRGPU_MXH_NT=$nt timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > $O/b${nt}_$rep.log 2>&1 || { tail -5 $O/b${nt}_$rep.log; exit 2; }
echo "nt=$nt rep=$rep $(tail -1 $O/b${nt}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
done
for nt in 3 7; do
SDRGPU_MXH_NT=$nt timeout -k 10 300 python bench_configs.py --config c5 --no-cpu-baseline > $O/c5_$nt.log 2>&1 || { tail -5 $O/c5_$nt.log; exit 3; }
echo "c5 nt=$nt $(tail -1 $O/c5_$nt.log | cut -c1-300)"
SDRGPU_MXH_NT=$nt timeout -k 10 300 python bench_configs.py --config c2u8 --no-cpu-baseline > $O/u8_$nt.log 2>&1 || { tail -5 $O/u8_$nt.log; exit 4; }
echo "u8 nt=$nt $(tail -1 $O/u8_$nt.log | cut -c1-300)"
done
