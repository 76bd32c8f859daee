#!/bin/bash
# PMC passes on the LDS-staged MFMA FIR kernel for the full kernel and its ablations.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_mxl
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
for abl in ${ABLS:-0 2 1}; do
  i=0
  for set in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
    i=$((i+1))
    SDRGPU_MX_ABLATION=$abl timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/a${abl}_p$i -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --algo mx > $O/a${abl}_p$i.log 2>&1 || { echo "abl $abl pass $i failed"; tail -5 $O/a${abl}_p$i.log; exit 1; }
  done
done
echo done
