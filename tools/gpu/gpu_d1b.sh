#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/d1b
mkdir -p $O
cd $R
for a in 1 2; do
SDRGPU_MX_ABLATION=$a timeout -k 10 300 python bench_configs.py --config c5 --no-cpu-baseline > $O/c5_a$a.log 2>&1 || { tail -5 $O/c5_a$a.log; exit 2; }
echo "abl $a $(tail -1 $O/c5_a$a.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline_rank0"]["kernel_ms"])')"
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc -o run -- python $R/bench_configs.py --config c5 --no-cpu-baseline --steps 2 > $O/pmc.log 2>&1 || { tail -3 $O/pmc.log; exit 3; }
python3 - <<'PY'
import csv,glob,collections
v=collections.defaultdict(list)
for f in glob.glob('/root/repo/gpurun_out/d1b/pmc/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        if 'mxh' in r['Kernel_Name']: v[r['Counter_Name']].append(float(r['Counter_Value']))
for k,x in sorted(v.items()): print(k, sum(x)/len(x))
PY
