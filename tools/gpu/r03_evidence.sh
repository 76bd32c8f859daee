#!/bin/bash
# Round-3 evidence pass: GPU tests, smoke, bench (+ rocprof stats), 2-rank bench rehearsal.
# Outputs under gpurun_out/$OUT/.  SKIP_TESTS=1 skips pytest.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_ev}
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cut -c1-900 $O/bench.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
cd $R
timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_2rank.jsonl 2> $O/bench_2rank.err || { tail -20 $O/bench_2rank.err; exit 9; }
cut -c1-1500 $O/bench_2rank.jsonl
