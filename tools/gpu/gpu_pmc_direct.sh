#!/bin/bash
# PMC passes (separate, --pmc only) over the default bench command for one algorithm.
# usage: gpu_pmc_direct.sh <algo> <outdir>
set -o pipefail
export OSV=${3:-1}
R=$GRAFT_REPO_ROOT
ALGO=${1:-direct}
OUT=$R/gpurun_out/${2:-pmc_direct}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  SDRGPU_OS_VARIANT=${OSV:-1} timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --algo $ALGO > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
