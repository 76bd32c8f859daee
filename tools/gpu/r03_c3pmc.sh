#!/bin/bash
# PMC passes over configs[2] (bench_configs c3, 2 steps) for one SDRGPU_F64X* variant ($V = "ns c w cb l").
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_c3pmc}
mkdir -p $O
cd $R
read -r ns c w cb l <<< "$V"; [ -n "$ENVX" ] && export $ENVX
export SDRGPU_F64X=$ns SDRGPU_F64X_C=$c SDRGPU_F64X_W=$w SDRGPU_F64X_CB=$cb SDRGPU_F64X_L=$l
export TMPDIR=/tmp
cd /tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $O/p$i -o run -- python3 $R/bench_configs.py --config c3 --no-cpu-baseline --no-check --steps 2 --warmup 1 > $O/p$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -5 $O/p$i.log; exit 1; }
done <<'EOC'
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT
EOC
cd $R
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt | head -40
