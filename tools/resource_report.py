"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one row per kernel.

usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/resource_report.py [filter]
"""
import re
import subprocess
import sys

rows, cur = [], None
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for line in sys.stdin:
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
print(f"{'kernel':60s} {'VGPR':>5s} {'spill':>5s} {'LDS':>6s} {'occ':>4s}")
for r, n in zip(rows, names):
    n = n.replace("void gd::", "").replace("(gd::Args)", "")
    if flt in n:
        print(f"{n:60s} {r.get('VGPRs','?'):>5s} {r.get('VGPRs Spill','?'):>5s} {r.get('LDS Size [bytes/block]','?'):>6s} {r.get('Occupancy [waves/SIMD]','?'):>4s}")
