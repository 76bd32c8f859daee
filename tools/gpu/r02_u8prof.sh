#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/u8prof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/bench_configs.py --config c2u8 --no-cpu-baseline > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/t/**/*kernel_stats.csv', recursive=True)[0])): print(r['Name'][:90], r['Calls'], r['AverageNs'])"
