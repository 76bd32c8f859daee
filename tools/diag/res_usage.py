"""Print VGPRs / AGPRs / spills / LDS per kernel from hipcc -Rpass-analysis=kernel-resource-usage
output: python tools/diag/res_usage.py FILE.res [name-substring]"""
import re
import sys

cur, rows = None, {}
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in rows.items():
    if pat in k:
        print(k[:90], v)
