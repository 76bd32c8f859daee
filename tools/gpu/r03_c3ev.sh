#!/bin/bash
# configs[2] evidence: rocprof kernel stats of bench_configs c3 (20 steps)
# and FETCH_SIZE / WRITE_SIZE passes (2 steps), summaries under gpurun_out/$OUT/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_c3bfp}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench_configs.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/p$i -o run -- python3 $R/bench_configs.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > $O/p$i.log 2>&1 || { echo "pass $i ($ctr) failed"; tail -5 $O/p$i.log; exit 2; }
done
cd $R
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; grep -A3 "fft64k" $O/summary.txt | head -20
grep -h "fft64k" $O/prof/run_kernel_stats.csv | cut -c1-160
