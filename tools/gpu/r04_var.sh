#!/bin/bash
# Round 4: driver-window / steady-state A/B of fir_ablate.sh variants (built here on the box)
# against the product library, REPS alternations of tools/gpu/r04_series.py --kind $KIND.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_var}
mkdir -p $O
cd $R
BUILD=$(echo $VARIANTS | tr " " "\n" | grep -v "^base$" | tr "\n" " ")
[ -z "$BUILD" ] || [ -n "$NOBUILD" ] || MAKEFLAGS=-j16 VARIANTS="$BUILD" timeout -k 10 600 bash tools/experiments/fir_ablate.sh > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
for rep in $(seq 1 ${REPS:-3}); do
  for v in prod $VARIANTS; do
    for kind in ${KINDS:-c64}; do
      f=$O/${v}_${kind}_$rep
      if [ $v = base ]; then
        timeout -k 10 120 python -u tools/experiments/run_with_lib.py tools/experiments/ab/lib_base.so tools/gpu/r04_series.py --kind $kind --long 200 > $f.jsonl 2> $f.err || { tail -20 $f.err; exit 2; }
      elif [ $v = prod ]; then
        timeout -k 10 120 python -u tools/gpu/r04_series.py --kind $kind --long 200 > $f.jsonl 2> $f.err || { tail -20 $f.err; exit 2; }
      else
        timeout -k 10 120 python -u tools/experiments/run_with_lib.py tools/experiments/abl/lib_$v.so tools/gpu/r04_series.py --kind $kind --long 200 > $f.jsonl 2> $f.err || { tail -20 $f.err; exit 2; }
      fi
    done
  done
done
python3 - $O <<'PY'
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for p in sorted(glob.glob(os.path.join(sys.argv[1], "*.jsonl"))):
    v, kind, rep = os.path.basename(p)[:-6].rsplit("_", 2)
    for l in open(p):
        d = json.loads(l)
        if d.get("phase") == "driver": acc[(kind, v, "1 driver(6-25)")].append(d["timed_mean"])
        if d.get("phase") == "long": acc[(kind, v, "2 steady")].append(d["mean"])
        if d.get("phase") == "idle": acc[(kind, v, "3 idle(6-25)")].append(sum(d["ms"][5:25]) / 20)
for k in sorted(acc, key=lambda k: (k[0], k[2], k[1])):
    print("%-5s %-14s %-16s" % (k[0], k[2], k[1]), " ".join("%.4f" % x for x in acc[k]), " mean %.4f" % (sum(acc[k]) / len(acc[k])))
PY
