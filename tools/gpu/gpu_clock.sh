#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/clock
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in 1 7 8; do
  SDRGPU_OS_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/v$v -o run -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --algo os > $OUT/v$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/v$v.log; exit 1; }
  SDRGPU_OS_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$v -o run -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --algo os > $OUT/t$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo done
