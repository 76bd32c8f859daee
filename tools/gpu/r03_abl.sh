#!/bin/bash
# headline FIR (bench.py kernel_ms) and configs[4] D=1 bank (bench_configs c5) under ablation
# libraries from tools/experiments/fir_ablate.sh ($LIBS: variant names; "base" = product lib).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_abl}
mkdir -p $O
cd $R
for v in ${LIBS:-base}; do
  if [ $v = base ]; then run="python"; else run="python tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so"; fi
  for rep in ${REPS:-1}; do
  timeout -k 10 120 $run bench.py --no-cpu-baseline --no-channel-sharded --steps 20 --warmup 3 > $O/fir_$v.$rep.jsonl 2> $O/fir_$v.$rep.err || { echo "fir $v failed"; tail -3 $O/fir_$v.$rep.err; exit 1; }
  timeout -k 10 120 $run bench_configs.py --config c5 --no-cpu-baseline --no-check --steps 10 --warmup 2 > $O/c5_$v.$rep.jsonl 2> $O/c5_$v.$rep.err || { echo "c5 $v failed"; tail -3 $O/c5_$v.$rep.err; exit 1; }
  python -c "
import json
f=json.loads(open('$O/fir_$v.$rep.jsonl').read().splitlines()[-1]); c=json.loads(open('$O/c5_$v.$rep.jsonl').read().splitlines()[-1])
print('$v', 'fir kernel_ms', f['roofline'].get('kernel_ms'), 'frac', f['roofline']['frac'], '| c5 ms', c['resident']['ms_per_step'], 'frac', c['resident']['roofline_frac_per_gpu'])"
  done
done
