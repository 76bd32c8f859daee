#!/bin/bash
# rocprof kernel stats for the session-4 kernels: examples' FFT shapes (gen_fixed_kernel) and
# the configs[3] PLL (pll_split_kernel, 2^18 samples per channel).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_new
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ex -o run -- python3 $R/bench_configs.py --config ex --no-cpu-baseline > $O/ex.log 2>&1 || { tail -5 $O/ex.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 $R/bench_configs.py --config c4 --no-cpu-baseline --c4-log2n 18 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 2; }
for d in ex c4; do python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/$d/**/*kernel_stats.csv', recursive=True)[0])): print('$d', r['Name'][:80], r['Calls'], r['AverageNs'])"; done
