#!/bin/bash
# Round 6: per-dispatch cycle / wait counters of the headline launch over a long bench run, to
# compare the driver's window (launches 6-25) with steady state (tools/pmc_window.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_pmc_window}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-channel-sharded > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
cd $R
python3 tools/pmc_window.py $O/p1 fir_mxh > $O/summary.txt 2>&1; cat $O/summary.txt
