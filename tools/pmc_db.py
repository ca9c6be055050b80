"""Per-kernel SQ / TCC counter sums from a rocprofv3 results database (--pmc ... -o <name>, default
sqlite output): python tools/pmc_db.py <results.db> [kernel-substring]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
q = "select kernel_name, dispatch_id, counter_name, sum(value) from counters_collection group by dispatch_id, counter_name"
per = collections.defaultdict(lambda: collections.defaultdict(list))
for k, d, n, v in c.execute(q):
    if flt in k:
        per[k.split("(")[0]][n].append(v)
for k, cs in per.items():
    print(k)
    for n, vs in sorted(cs.items()):
        print(f"    {n:28s} mean over {len(vs):3d} dispatches {sum(vs) / len(vs):16.1f}")
