#!/bin/bash
# Round 4: which part of the headline launch sets its clock dip -- clk-stamped ablations
# (tools/experiments/fir_ablate.sh composite variants, built on the box) through
# tools/gpu/r04_series.py --clk, alternating REPS times.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_dip2}
mkdir -p $O
cd $R
VS="${VARIANTS:-clk clk+nomfma clk+noload clk+mfma4 clk+nosplit}"
MAKEFLAGS=-j16 VARIANTS="$VS" timeout -k 10 600 bash tools/experiments/fir_ablate.sh > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
L=tools/experiments/abl
for rep in $(seq 1 ${REPS:-1}); do
for v in $VS; do
  for kind in ${KINDS:-c64}; do
    timeout -k 10 120 python -u tools/experiments/run_with_lib.py $L/lib_$v.so tools/gpu/r04_series.py --kind $kind --clk --long ${LONG:-200} > $O/${v}_${kind}_$rep.jsonl 2> $O/${v}_${kind}_$rep.err || { tail -20 $O/${v}_${kind}_$rep.err; exit 2; }
  done
done
done
python3 - $O <<'PY'
import glob, json, os, sys
for p in sorted(glob.glob(os.path.join(sys.argv[1], "*.jsonl"))):
    for l in open(p):
        d = json.loads(l)
        if "ms" not in d:
            continue
        ms, mhz = d["ms"], d.get("mhz") or [0] * len(d["ms"])
        mhz = [m or 0 for m in mhz]
        line = f"{os.path.basename(p):28s} {d['phase']:6s} mean {d['mean']:.4f} first6 {sum(ms[:6])/6:.4f} mid(6-15) {sum(ms[6:16])/10:.4f} last10 {sum(ms[-10:])/10:.4f}"
        if d.get("timed_mean"): line += f" timed {d['timed_mean']:.4f}"
        line += f" | MHz first6 {sum(mhz[:6])/6:.0f} min {min(mhz[1:]):.0f} mid {sum(mhz[6:16])/10:.0f} last10 {sum(mhz[-10:])/10:.0f}"
        print(line)
PY
