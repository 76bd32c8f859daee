import csv, sys, glob, collections
d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ''
vals = collections.defaultdict(list)
for f in glob.glob(d + '/p*/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if pat and pat not in row['Kernel_Name']:
            continue
        vals[row['Counter_Name']].append(float(row['Counter_Value']))
for k, v in sorted(vals.items()):
    # rows are per-dispatch (summed over dimensions?) -> report mean per dispatch
    print(f"{k:28s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
