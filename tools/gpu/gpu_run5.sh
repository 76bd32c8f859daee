#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
case "$(tail -1 gpurun_out/pytest_gpu.log)" in *"rc=0"|*"rc=1") ;; *) echo "pytest died"; exit 1;; esac
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_v2
cd /tmp
i=0
for set in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_v2/p$i -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --algo os > $R/gpurun_out/pmc_v2/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
