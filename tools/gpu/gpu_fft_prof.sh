#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fftprof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench_configs.py --config c3 --steps 3 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cut -c1-160 $O/trace/run_kernel_stats.csv | head -6
