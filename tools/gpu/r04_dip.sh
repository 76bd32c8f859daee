#!/bin/bash
# Round 4: per-launch series (tools/gpu/r04_series.py) of the product FIR launches and of the
# clk / nomfma / noload builds (tools/experiments/fir_ablate.sh, built here on the box), for
# the headline (c64), the rtl_tcp u8 launch and the configs[4] D = 1 bank.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_dip}
mkdir -p $O
cd $R
MAKEFLAGS=-j16 VARIANTS="${VARIANTS:-clk nomfma noload}" timeout -k 10 400 bash tools/experiments/fir_ablate.sh > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
L=tools/experiments/abl
for kind in ${KINDS:-c64 u8 bank}; do
  timeout -k 10 120 python -u tools/gpu/r04_series.py --kind $kind > $O/prod_$kind.jsonl 2> $O/prod_$kind.err || { tail -20 $O/prod_$kind.err; exit 2; }
  timeout -k 10 120 python -u tools/experiments/run_with_lib.py $L/lib_clk.so tools/gpu/r04_series.py --kind $kind --clk > $O/clk_$kind.jsonl 2> $O/clk_$kind.err || { tail -20 $O/clk_$kind.err; exit 3; }
  for v in nomfma noload; do
    [ -f $L/lib_$v.so ] || continue
    timeout -k 10 120 python -u tools/experiments/run_with_lib.py $L/lib_$v.so tools/gpu/r04_series.py --kind $kind > $O/${v}_$kind.jsonl 2> $O/${v}_$kind.err || { tail -20 $O/${v}_$kind.err; exit 4; }
  done
done
python3 - $O <<'PY'
import glob, json, os, sys
for p in sorted(glob.glob(os.path.join(sys.argv[1], "*.jsonl"))):
    for l in open(p):
        d = json.loads(l)
        if "ms" not in d:
            continue
        ms = d["ms"]
        mhz = d.get("mhz")
        line = f"{os.path.basename(p):22s} {d['phase']:6s} mean {d['mean']:.4f} first6 {sum(ms[:6])/6:.4f} "
        line += f"mid(6-15) {sum(ms[6:16])/10:.4f} last10 {sum(ms[-10:])/10:.4f}"
        if d.get("timed_mean"): line += f" timed {d['timed_mean']:.4f}"
        if mhz: line += f" MHz first6 {sum(mhz[:6])/6:.0f} mid {sum(mhz[6:16])/10:.0f} last10 {sum(mhz[-10:])/10:.0f}"
        print(line)
PY
