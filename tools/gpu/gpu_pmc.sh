#!/bin/bash
# PMC passes on the FIR kernel (bench.py, 2^28 samples, 3 steps). Counters per pass kept small.
set -o pipefail
R=$GRAFT_REPO_ROOT
ALGO=${1:-os}
mkdir -p $R/gpurun_out/pmc_$ALGO
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $R/gpurun_out/pmc_$ALGO/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_$ALGO/p$i -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --algo $ALGO > $R/gpurun_out/pmc_$ALGO/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
