#!/bin/bash
# Steady-state A/B of tools/experiments/abl/lib_<v>.so variants against libbase.so on one box:
# REPS rounds, each running base then every variant in VARIANTS through
# `bench.py --no-cpu-baseline --no-channel-sharded` (200 steps).  Logs under gpurun_out/$OUT/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_var}
mkdir -p $O
cd $R
SCRIPT=${SCRIPT:-"bench.py --no-cpu-baseline --no-channel-sharded"}
for i in $(seq 1 ${REPS:-2}); do
  for v in base $VARIANTS; do
    if [ $v = base ]; then L=tools/experiments/abl/libbase.so; else L=tools/experiments/abl/lib_$v.so; fi
    timeout -k 10 300 python tools/experiments/run_with_lib.py $L $SCRIPT > $O/$v.$i.jsonl 2> $O/$v.$i.err || { tail -20 $O/$v.$i.err; exit 3; }
    echo "$v $i $(python -c "
import json
for l in open('$O/$v.$i.jsonl'):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l); r=d.get('roofline',{}); c=d.get('channel_sharded',{}).get('resident',{})
    w=d.get('config',{}); w=w.get('workload','') if isinstance(w,dict) else w
    print(w[:12], r.get('kernel_ms'), r.get('frac'), 'c5', c.get('ms_per_step'), c.get('roofline_frac_per_gpu'))
")" | tee -a $O/summary.txt
  done
done
