"""Summarise rocprofv3 --pmc counter CSVs: per kernel, per counter, the mean over dispatches
of the per-dispatch total (rows of one dispatch are summed).  Usage: pmc_summary.py DIR [substr]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ''
per = collections.defaultdict(float)           # (kernel, counter, dispatch) -> value
for f in glob.glob(d + '/p*/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        k = row['Kernel_Name']
        if pat and pat not in k:
            continue
        per[(k[:90], row['Counter_Name'], row.get('Dispatch_Id', '0'))] += float(row['Counter_Value'])
agg = collections.defaultdict(list)
for (k, c, _), v in per.items():
    agg[(k, c)].append(v)
for (k, c), v in sorted(agg.items()):
    print(f"{k:90s} {c:22s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
