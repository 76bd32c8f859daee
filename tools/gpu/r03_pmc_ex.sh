#!/bin/bash
# examples/live.rs STFT shape (gen_tile_kernel): SQ / LDS / memory counters, one pass each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-pmc_live}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() {
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/p$n -o run -- python3 $R/bench_configs.py --config ex --no-cpu-baseline --steps 3 --warmup 1 > $O/p$n.log 2>&1 || { tail -5 $O/p$n.log; exit $n; }
}
run 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD
run 2 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
run 3 FETCH_SIZE
run 4 WRITE_SIZE
python3 $R/tools/pmc_summary.py $O gen_ > $O/summary.txt; cat $O/summary.txt
