#!/bin/bash
# Round 4: the driver's bench command with one event pair around the timed launches (now) vs
# an event pair around every launch (--event-per-launch, rounds 1-4), alternating, then a
# rocprofv3 kernel trace of the driver's command (gaps between the timed launches).
# Ran against a bench.py with the one-pair timing and an --event-per-launch flag (round 4);
# the one-pair variant was not kept, so bench.py has neither the mode nor the flag now
# (result: profiles/r04_bench_timing_ab.txt).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_timing}
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for m in one per; do
    f=$O/bench_${m}_$rep.jsonl
    if [ $m = per ]; then X=--event-per-launch; else X=; fi
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-channel-sharded $X > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$f').readline()); print('$m', $rep, d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.jsonl 2> $O/prof.log || { tail -20 $O/prof.log; exit 4; }
cut -c1-300 $O/prof.jsonl
