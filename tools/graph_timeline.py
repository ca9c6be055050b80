"""Per-replay kernel timeline from a rocprofv3 kernel trace of tools/graph_trace.py: the last R replays
(each the same sequence of dispatches as the final one), per position the mean duration and the mean gap
from the previous kernel's end (position 0: from the previous replay's last kernel).

usage: python tools/graph_timeline.py <kernel_trace.csv> <kernels per replay, 0 = detect> [R]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = int(sys.argv[2])
R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if per == 0:  # the shortest period of the kernel-name sequence over the trace's tail
    nm = [r["Kernel_Name"] for r in rows[-400:]]
    per = next(p for p in range(1, len(nm) // 3) if all(nm[-1 - i] == nm[-1 - i - p] for i in range(2 * p)))
rows = rows[-per * R:]
n = len(rows) // per
dur = [0.0] * per
gap = [0.0] * per
names = [""] * per
tot = []
for rep in range(n):
    seq = rows[rep * per:(rep + 1) * per]
    for i, r in enumerate(seq):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[i] += (e - s) / 1e3
        if i > 0:
            gap[i] += (s - int(seq[i - 1]["End_Timestamp"])) / 1e3
        elif rep > 0:
            gap[i] += (s - int(rows[rep * per - 1]["End_Timestamp"])) / 1e3
        names[i] = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]
    tot.append((int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3)
print(f"{n} replays, {per} kernels each; first-start -> last-end {sum(tot) / n:.1f} us")
for i in range(per):
    print(f"{i:3d} {names[i]:60s} {dur[i] / n:8.2f} us  gap before {gap[i] / max(1, n - (i == 0)):7.2f} us")
print(f"sum of kernels {sum(dur) / n:.1f} us, sum of gaps {sum(gap[1:]) / n:.1f} us (+ {gap[0] / max(1, n - 1):.1f} between replays)")
