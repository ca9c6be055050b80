"""Per-kernel means of rocprofv3 --pmc SQ counters (csv output), summed over a dispatch's instances.

usage: python tools/sq_summary.py <counter_collection.csv> [<counter_collection.csv> ...]
"""
import collections
import csv
import re
import sys

per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter -> sum
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = re.sub(r"\(.*", "", r.get("Kernel_Name", "")).replace("void ", "")
        per[(k, path, r.get("Dispatch_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (k, _, _), cs in per.items():
    for n, v in cs.items():
        agg[k][n].append(v)
for k, cs in sorted(agg.items()):
    print(k)
    for n, vs in sorted(cs.items()):
        print(f"    {n:24s} mean over {len(vs):3d} dispatches {sum(vs) / len(vs):16.1f}")
    m = {n: sum(vs) / len(vs) for n, vs in cs.items()}
    if m.get("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        print(f"    -> VALU active {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}, any-inst active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}, "
              f"waiting {m.get('SQ_WAIT_ANY', 0) / wc:.3f} (of wave cycles)")
    if m.get("SQ_LDS_IDX_ACTIVE"):
        print(f"    -> LDS bank-conflict cycles / LDS cycles {m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.3f}")
