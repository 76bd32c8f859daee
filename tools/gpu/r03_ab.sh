#!/bin/bash
# A/B of the product library against tools/experiments/abl/libbase.so on one box:
# optional pytest subset (TESTS="tests/test_fir_gpu.py ..."), then REPS alternating runs of
# SCRIPT (default bench.py --no-cpu-baseline) with each library.  Logs under gpurun_out/$OUT/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_ab}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
SCRIPT=${SCRIPT:-"bench.py --no-cpu-baseline"}
for i in $(seq 1 ${REPS:-2}); do
  for v in base new; do
    if [ $v = base ]; then L=tools/experiments/abl/libbase.so; else L=unnamed-rust-sdr_amd/libsdrgpu.so; fi
    timeout -k 10 300 python tools/experiments/run_with_lib.py $L $SCRIPT > $O/$v.$i.jsonl 2> $O/$v.$i.err || { tail -20 $O/$v.$i.err; exit 3; }
    echo "$v $i $(python -c "
import json,sys
for l in open('$O/$v.$i.jsonl'):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l); r=d.get('roofline',{}); c=d.get('channel_sharded',{}).get('resident',{})
    print(d.get('config',{}).get('workload','')[:12], r.get('kernel_ms'), r.get('frac'), 'c5', c.get('ms_per_step'), c.get('roofline_frac_per_gpu'))
")"
  done
done
