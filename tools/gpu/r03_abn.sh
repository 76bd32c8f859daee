#!/bin/bash
# Alternating bench runs of several libraries: LIBS="name=path ..." REPS=n SCRIPT="bench.py ...".
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_abn}
mkdir -p $O
cd $R
SCRIPT=${SCRIPT:-"bench.py --no-cpu-baseline"}
for i in $(seq 1 ${REPS:-2}); do
  for nl in $LIBS; do
    v=${nl%%=*}; L=${nl#*=}
    timeout -k 10 300 python tools/experiments/run_with_lib.py $L $SCRIPT > $O/$v.$i.jsonl 2> $O/$v.$i.err || { tail -20 $O/$v.$i.err; exit 3; }
    echo "$v $i $(python -c "
import json
for l in open('$O/$v.$i.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); r=d.get('roofline',{}); c=d.get('channel_sharded',{}).get('resident',{})
        print(r.get('kernel_ms'), r.get('frac'), 'c5', c.get('ms_per_step'), c.get('roofline_frac_per_gpu'))
")"
  done
done
