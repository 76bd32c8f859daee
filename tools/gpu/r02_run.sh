#!/bin/bash
# run-interleaved units (SDRGPU_TMP_RUN = tiles per run): parity then c2 / c5 / c2u8 A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run
mkdir -p $O
cd $GRAFT_REPO_ROOT
for run in 0 4 16; do
SDRGPU_TMP_RUN=$run timeout -k 10 300 python -u -m pytest tests/test_firbank_gpu.py tests/test_fir_gpu.py tests/test_ingest_gpu.py tests/test_signal.py tests/test_stream_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_$run.log 2>&1 || { tail -30 $O/pytest_$run.log; exit 1; }
echo "run=$run $(tail -1 $O/pytest_$run.log)"
done
for rep in 1 2; do
  for run in 0 2 4 8 16; do
    SDRGPU_TMP_RUN=$run timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 > $O/b_${run}_${rep}.log 2>&1 || exit 2
    echo "c2 run=$run rep=$rep $(tail -1 $O/b_${run}_${rep}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
for run in 0 4 16; do
  SDRGPU_TMP_RUN=$run timeout -k 10 200 python bench_configs.py --config c5 --no-cpu-baseline > $O/c5_$run.log 2>&1 || exit 3
  echo "c5 run=$run $(tail -1 $O/c5_$run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline_rank0"]; print(r["kernel_ms"], r["frac"])')"
  SDRGPU_TMP_RUN=$run timeout -k 10 200 python bench_configs.py --config c2u8 > $O/u8_$run.log 2>&1 || exit 4
  echo "c2u8 run=$run $(tail -1 $O/u8_$run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms"], r["frac"])')"
done
