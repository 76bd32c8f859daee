#!/bin/bash
# Round 4: instruction-mix PMC passes (one counter group per rocprofv3 run, each under its own
# timeout) over `bench.py --steps 20 --warmup 5` (headline leg only), optionally against a
# variant library: LIB=tools/experiments/abl/lib_<v>.so.  r04_pmc.sh <outdir>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04_pmc}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
if [ -n "$LIB" ]; then RUN="$R/tools/experiments/run_with_lib.py $R/$LIB $R/bench.py"; else RUN="$R/bench.py"; fi
timeout -k 10 -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 $RUN --steps 20 --warmup 5 --no-cpu-baseline --no-channel-sharded > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python3 $R/tools/pmc_summary.py $O > $O/summary.txt 2>&1; grep fir_mxh $O/summary.txt | sed 's/^.\{90\}//'
