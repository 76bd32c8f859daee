"""Per-dispatch PMC counters of one kernel in launch order (rocprofv3 --kernel-trace --pmc CSVs):
means over launches 6-25 of the run (bench.py's driver window) and over the last 100, per
counter, plus the kernel duration and the effective clock GRBM_GUI_ACTIVE / 8 / duration.
Usage: pmc_window.py DIR kernel-substring"""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(float))   # dispatch -> counter -> sum
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if pat in row['Kernel_Name']:
            vals[int(row['Dispatch_Id'])][row['Counter_Name']] += float(row['Counter_Value'])
dur = {}
for f in glob.glob(d + '/**/*kernel_trace.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if pat in row['Kernel_Name']:
            dur[int(row['Dispatch_Id'])] = (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) * 1e-6
ids = sorted(vals)
print(f"{len(ids)} dispatches of *{pat}*; durations for {len(dur)}")
groups = {"window (launches 6-25)": ids[5:25], "steady (last 100)": ids[-100:]}
counters = sorted({c for i in ids for c in vals[i]})
for name, sel in groups.items():
    print(f"== {name}: n = {len(sel)}")
    ms = [dur[i] for i in sel if i in dur]
    if ms:
        print(f"  duration_ms {sum(ms) / len(ms):.4f}")
    for c in counters:
        v = [vals[i][c] for i in sel]
        print(f"  {c:26s} {sum(v) / len(v):.6g}")
    if ms and all('GRBM_GUI_ACTIVE' in vals[i] for i in sel):
        clk = [vals[i]['GRBM_GUI_ACTIVE'] / 8 / (dur[i] * 1e-3) / 1e9 for i in sel if i in dur]
        print(f"  effective clock GHz (GRBM_GUI_ACTIVE / 8 / duration) {sum(clk) / len(clk):.3f}")
