#!/bin/bash
# Batched SincFastest wide-frame kernel: SQ / LDS / L2 counters, one pass each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_sinc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() {
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/p$n -o run -- python3 $R/bench_configs.py --config src --no-cpu-baseline > $O/p$n.log 2>&1 || { tail -5 $O/p$n.log; exit $n; }
}
run 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
run 2 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE
run 3 TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
python3 $R/tools/pmc_summary.py $O src_sinc_wide > $O/summary.txt; cat $O/summary.txt
