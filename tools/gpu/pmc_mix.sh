#!/bin/bash
# Instruction-mix PMC passes (one counter group per rocprofv3 run, each under its own timeout)
# over a command that launches the kernel of interest, optionally against a variant library
# (LIB=...so).  pmc_mix.sh <outdir> <kernel-substring> <script> [args...]
#   tools/gpu/pmc_mix.sh r05_pmc_bank fir_mxh bench_configs.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-check
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1; K=$2; shift 2
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
if [ -n "$LIB" ]; then RUN="$R/tools/experiments/run_with_lib.py $R/$LIB $R/$1"; else RUN="$R/$1"; fi
shift
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 $RUN "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O $K > $O/summary.txt 2>&1; sed 's/^.\{60\}//' $O/summary.txt
