#!/bin/bash
# kernel trace of the resampler bench lines (per-kernel durations)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/src_prof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/bench_configs.py --config src --no-cpu-baseline > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
f=$(find $O/t -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | cut -c1-160
