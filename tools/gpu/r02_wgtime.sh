#!/bin/bash
# Tail census of the headline FIR: per-workgroup start/end times (fir_ablate.sh wgtime).
set -o pipefail
O=gpurun_out/wgtime
mkdir -p $O
timeout -k 10 120 python tools/experiments/run_with_lib.py tools/experiments/abl/lib_wgtime.so tools/experiments/fir_tail.py > $O/run.txt 2>&1 || { tail -5 $O/run.txt; exit 1; }
cat $O/run.txt
exit 0
python3 - <<'PY'
import collections
rows = [l.split() for l in open('gpurun_out/wgtime/run.txt') if l.startswith('WGT')]
# group launches: 256 lines each, in order of appearance is not guaranteed -> group by start time clusters
rows = [(int(b), int(x), int(s), int(e)) for _, b, x, s, e in rows]
rows.sort(key=lambda r: r[2])
launches = []
cur = []
for r in rows:
    if cur and r[2] - cur[0][2] > 20000:  # > 200 us after the first start: next launch
        launches.append(cur); cur = []
    cur.append(r)
if cur: launches.append(cur)
for L in launches:
    s0 = min(r[2] for r in L); e1 = max(r[3] for r in L)
    ends = sorted((r[3] - s0) / 100.0 for r in L)  # us
    starts = sorted((r[2] - s0) / 100.0 for r in L)
    byx = collections.defaultdict(list)
    for r in L: byx[r[1]].append((r[3] - s0) / 100.0)
    print(f"launch n={len(L)} span {(e1 - s0) / 100.0:.1f} us; start spread {starts[-1]:.1f} us; "
          f"end min/p10/p50/p90/max {ends[0]:.1f}/{ends[len(ends)//10]:.1f}/{ends[len(ends)//2]:.1f}/{ends[9*len(ends)//10]:.1f}/{ends[-1]:.1f} us")
    print("   per-XCD mean end:", " ".join(f"{x}:{sum(v)/len(v):.1f}" for x, v in sorted(byx.items())))
PY
grep '^{' $O/run.txt | cut -c1-200
