"""Count instruction classes in a kernel's hottest loop (the largest block range that ends in
a backward branch) of a hipcc -save-temps .s file.
Usage: isa_count.py FILE.s KERNEL_SUBSTRING [samples_per_iteration]"""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], sys.argv[2]
per = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
src = open(path).read().splitlines()
start = next(i for i, l in enumerate(src) if re.match(r'^_Z\S*:', l) and pat in l)
end = next(i for i in range(start, len(src)) if src[i].startswith('.Lfunc_end'))
body = src[start:end]
labels = {l.split(':')[0]: i for i, l in enumerate(body) if re.match(r'^\.LBB\S+:', l)}
best = None
for i, l in enumerate(body):
    m = re.match(r'\s+s_cbranch_\w+\s+(\.LBB\S+)|\s+s_branch\s+(\.LBB\S+)', l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            if best is None or i - labels[tgt] > best[1] - best[0]:
                best = (labels[tgt], i)
lo, hi = best
c = Counter()
for l in body[lo:hi + 1]:
    t = l.strip().split()
    if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
        continue
    op = t[0]
    if op.startswith('v_mfma'): c['mfma'] += 1
    elif op.startswith(('v_div_scale', 'v_div_fmas', 'v_div_fixup')): c['valu_div'] += 1; c['valu'] += 1
    elif op.startswith(('v_readlane', 'v_writelane', 'v_readfirstlane')): c['lane_xfer'] += 1
    elif op.endswith('_f64'): c['valu_f64'] += 1; c['valu'] += 1
    elif op.startswith('v_'): c['valu'] += 1
    elif op.startswith('s_cbranch'): c['cbranch'] += 1
    elif op.startswith('s_waitcnt'): c['waitcnt'] += 1
    elif op.startswith('s_'): c['salu'] += 1
    elif op.startswith(('global_load', 'buffer_load', 'flat_load')): c['vmem_load'] += 1
    elif op.startswith(('global_store', 'buffer_store', 'flat_store')): c['vmem_store'] += 1
    elif op.startswith('ds_'): c['lds'] += 1
    else: c['other:' + op] += 1
print(f"loop lines {lo}-{hi} of {pat}:")
for k, v in sorted(c.items()):
    print(f"  {k:12s} {v:6d}  ({v / per:.1f} per sample)")
