#!/bin/bash
# Sinc resampler: GPU parity (bit-exact vs the oracle) + bench lines.
set -o pipefail
O=gpurun_out/sinc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resample.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench_configs.py --config src --no-cpu-baseline > $O/src.jsonl 2> $O/src.err || { tail -20 $O/src.err; exit 2; }
cut -c1-400 $O/src.jsonl
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/t -o run -- python3 $GRAFT_REPO_ROOT/bench_configs.py --config src --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/t.log 2>&1) || exit 3
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob(\"$O/t/**/*kernel_stats.csv\", recursive=True)[0])): print(r[\"Name\"][:60], r[\"Calls\"], r[\"AverageNs\"])"
