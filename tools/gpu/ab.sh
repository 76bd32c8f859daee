#!/bin/bash
# A/B of the product library against a baseline build (BASE=path to a .so, default
# tools/diag/probe_build/lib_base.so: the previous build, copied there before the change;
# git-ignored, travels with the snapshot): REPS alternations of the per-launch series
# (tools/gpu/series.py --kind K for K in KINDS), summarised as driver-window (launches
# 6-25: what `bench.py --steps 20 --warmup 5` times) and steady-state (last 200) means.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-ab}
BASE=${BASE:-tools/diag/probe_build/lib_base.so}
mkdir -p $O
cd $R
# ARMS="name=lib.so ..." alternates several builds instead (names without "_"; "new" = product)
ARMS=${ARMS:-"base=$BASE new=product"}
for rep in $(seq 1 ${REPS:-3}); do
  for arm in $ARMS; do
    v=${arm%%=*}; lib=${arm#*=}
    for kind in ${KINDS:-c64}; do
      if [ $lib != product ]; then
        timeout -k 10 120 python -u tools/experiments/run_with_lib.py $lib tools/gpu/series.py --kind $kind --long 200 > $O/${v}_${kind}_$rep.jsonl 2> $O/${v}_${kind}_$rep.err || { tail -20 $O/${v}_${kind}_$rep.err; exit 2; }
      else
        timeout -k 10 120 python -u tools/gpu/series.py --kind $kind --long 200 > $O/${v}_${kind}_$rep.jsonl 2> $O/${v}_${kind}_$rep.err || { tail -20 $O/${v}_${kind}_$rep.err; exit 2; }
      fi
    done
  done
done
python3 - $O <<'PY'
import glob, json, os, sys, collections
acc = collections.defaultdict(list)
for p in sorted(glob.glob(os.path.join(sys.argv[1], "*.jsonl"))):
    v, kind, rep = os.path.basename(p)[:-6].split("_")
    for l in open(p):
        d = json.loads(l)
        if d.get("phase") == "driver": acc[(kind, v, "driver")].append(d["timed_mean"])
        if d.get("phase") == "long": acc[(kind, v, "steady")].append(d["mean"])
        if d.get("phase") == "idle": acc[(kind, v, "idle")].append(sum(d["ms"][5:25]) / 20)
for k in sorted(acc):
    print(k, " ".join("%.4f" % x for x in acc[k]), " mean %.4f" % (sum(acc[k]) / len(acc[k])))
PY
