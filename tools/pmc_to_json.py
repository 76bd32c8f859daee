"""Turn the FETCH_SIZE / WRITE_SIZE PMC passes of the default bench command into
profiles/pmc_fir_c2.json (read by bench.py as roofline.traffic).

gfx950 corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE counts half
the bytes of a coalesced streaming read -> x2; WRITE_SIZE is exact for streaming stores.
Both are reported in KiB per dispatch."""
import csv, glob, json, os, sys, collections

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_source_sha16: ties the figure to the kernel source)

def per_dispatch(d, counter, pat):
    vals = []
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for row in csv.DictReader(open(f)):
            if row['Counter_Name'] == counter and pat in row['Kernel_Name']:
                vals.append(float(row['Counter_Value']))
    return vals

src, out = sys.argv[1], sys.argv[2]
pat = sys.argv[3] if len(sys.argv) > 3 else 'fir_'
fe = per_dispatch(src + '/pmc_fetch', 'FETCH_SIZE', pat)
wr = per_dispatch(src + '/pmc_write', 'WRITE_SIZE', pat)
fetch = 2 * 1024 * max(fe)   # the timed launches; the tiny halo-priming launch is smaller
write = 1024 * max(wr)
res = {"log2n": 28, "algo": "auto", "kernel_pattern": pat,
       "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
       "hbm_bytes_per_launch": fetch + write,
       "dispatches": {"fetch": fe, "write": wr},
       "kernel_source_sha16": bench.kernel_source_sha16(),
       "kernel_sources": list(bench.KERNEL_SOURCES),
       "commit": os.environ.get("GIT_COMMIT"),
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                 "`python bench.py --steps 3 --warmup 1 --no-cpu-baseline`; FETCH_SIZE x2 (gfx950 "
                 "streaming-read correction), KiB -> bytes"}
json.dump(res, open(out, 'w'), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != 'dispatches'}))
