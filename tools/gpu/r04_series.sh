#!/bin/bash
# Round 4: per-launch series of the headline launch (tools/gpu/r04_series.py) and a
# per-dispatch rocprofv3 kernel trace of the driver's exact bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_series}
mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/gpu/r04_series.py > $O/series.jsonl 2> $O/series.err || { tail -20 $O/series.err; exit 1; }
python -c "
import json
for l in open('$O/series.jsonl'):
    d=json.loads(l); d.pop('ms',None); print(d)
"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o drv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.jsonl 2> $O/drv.err || { tail -20 $O/drv.err; exit 2; }
cut -c1-600 $O/drv.jsonl
cd $R
if [ -n "$EXTRA_TESTS" ]; then
timeout -k 10 600 python -u -m pytest $EXTRA_TESTS ${EXTRA_K:+-k "$EXTRA_K"} -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/extra_tests.log 2>&1 || { tail -30 $O/extra_tests.log; exit 3; }
tail -3 $O/extra_tests.log
fi
if [ -n "$C4" ]; then
timeout -k 10 300 python -u bench_configs.py --config c4 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 4; }
cut -c1-1200 $O/c4.jsonl
fi
if [ -n "$C3PAIR" ]; then
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -o /tmp/stft64k_pair tools/experiments/stft64k_pair.hip || exit 5
timeout -k 10 120 /tmp/stft64k_pair 20 > $O/c3pair.txt 2>&1; rc=$?; cat $O/c3pair.txt; [ $rc -le 2 ] || exit 6
fi
