"""Per-basic-block instruction mix of one kernel in a hipcc -save-temps .s file (diagnostic:
which blocks carry the MFMAs, the spills and the SALU).
usage: python tools/diag/isa_blocks.py FILE.s KERNEL_SYMBOL [min_instructions]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
name = sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
blocks, cur = [], ('entry', [])
for l in s[i:j].split('\n'):
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        blocks.append(cur)
        cur = (m.group(1), [])
        continue
    t = l.strip()
    if l.startswith('\t') and t and not t.startswith(('.', ';')):
        cur[1].append(t)
blocks.append(cur)


def cat(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op in ('v_readlane_b32', 'v_writelane_b32'):
        return 'lane'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_nop'):
        return 'nop'
    if op.startswith('s_waitcnt'):
        return 'wait'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_')):
        return 'vmem'
    return 'other'


for lab, ins in blocks:
    if len(ins) < mn:
        continue
    c = Counter(cat(x.split()[0]) for x in ins)
    br = [x for x in ins if x.startswith('s_cbranch') or x.startswith('s_branch')]
    print(f"{lab:14s} n={len(ins):4d} " + ' '.join(f"{k}={c[k]}" for k in
          ('mfma', 'valu', 'lane', 'salu', 'nop', 'wait', 'lds', 'vmem')) + '  ' + ' | '.join(br[-2:]))
