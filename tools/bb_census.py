"""Per-basic-block instruction census of one kernel in a hipcc -save-temps .s file: for every
block with more than MIN instructions, its MFMA / VALU / v_readlane+v_writelane (SGPR spill
traffic) / SALU / LDS / global counts -- to find the hot loop's blocks and what they carry.
Usage: bb_census.py FILE.s KERNEL_SUBSTRING [MIN]"""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
src = open(path).read().splitlines()
start = next(i for i, l in enumerate(src) if re.match(r'^_Z\S*:', l) and pat in l)
end = next(i for i in range(start, len(src)) if src[i].startswith('.Lfunc_end'))
blocks, cur = [], ['entry', start, []]
blocks.append(cur)
for i in range(start + 1, end):
    l = src[i]
    if re.match(r'^\.LBB\S+:', l):
        cur = [l.split(':')[0], i, []]
        blocks.append(cur)
        continue
    t = l.strip().split()
    if t and not t[0].startswith(('.', ';')) and not t[0].endswith(':'):
        cur[2].append(t[0])
for name, i, ins in blocks:
    if len(ins) <= mn:
        continue
    c = lambda f: sum(1 for x in ins if f(x))
    print(f"{name:14s} line {i:6d} n={len(ins):4d} mfma={c(lambda x: x.startswith('v_mfma')):3d} "
          f"valu={c(lambda x: x.startswith('v_') and not x.startswith(('v_mfma', 'v_readlane', 'v_writelane'))):4d} "
          f"lanex={c(lambda x: x.startswith(('v_readlane', 'v_writelane'))):3d} "
          f"salu={c(lambda x: x.startswith('s_') and not x.startswith(('s_waitcnt', 's_cbranch', 's_branch', 's_nop'))):4d} "
          f"ds={c(lambda x: x.startswith('ds_')):3d} gl={c(lambda x: x.startswith(('global_', 'buffer_'))):3d} "
          f"end={ins[-1]}")
