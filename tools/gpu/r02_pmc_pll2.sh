#!/bin/bash
# PLL PMC: one SQ pass over bench_configs c4 with the given library runner prefix
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/p1 -o run -- python3 "$@" > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
python3 $R/tools/pmc_summary.py $O pll_ > $O/summary.txt; cat $O/summary.txt
