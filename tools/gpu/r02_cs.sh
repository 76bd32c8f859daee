#!/bin/bash
# D=1 bank column sets per tile (CS) A/B: parity for CS=2,3 then c5 per CS
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/cs
mkdir -p $O
cd $GRAFT_REPO_ROOT
for cs in 2 3; do
  SDRGPU_TMP_CS1=$cs timeout -k 10 300 python -u -m pytest tests/test_firbank_gpu.py tests/test_fir_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_$cs.log 2>&1 || { tail -30 $O/pytest_$cs.log; exit 1; }
  echo "cs=$cs $(tail -1 $O/pytest_$cs.log)"
done
for rep in 1 2; do
  for cs in 1 2 3; do
    SDRGPU_TMP_CS1=$cs timeout -k 10 200 python bench_configs.py --config c5 --no-cpu-baseline > $O/c5_${cs}_$rep.log 2>&1 || exit 3
    echo "c5 cs=$cs rep=$rep $(tail -1 $O/c5_${cs}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline_rank0"]; print(r["kernel_ms"], r["frac"], d.get("spot_check_max_over_rms"))')"
  done
done
