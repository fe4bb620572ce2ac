"""Per-dispatch table of rocprofv3 --pmc counters (summed over dimensions), one row per (kernel, dispatch) of the
first run found for each counter pass, merged across passes by launch order of that kernel name.
usage: pmc_table.py <dir with p*/ rocprofv3 outputs> | <csv> [...]"""
import collections
import csv
import glob
import os
import re
import sys

paths = []
for a in sys.argv[1:]:
    paths += sorted(glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True)) if os.path.isdir(a) else [a]
rows = collections.defaultdict(dict)  # (kernel, k-th launch) -> counter -> value
for path in paths:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name_of = {}
    for r in csv.DictReader(open(path)):
        m = re.search(r"hyk::(\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        name_of[d] = name
    seen = collections.Counter()
    for d in sorted(per):
        k = name_of[d]
        rows[(k, seen[k])].update(per[d])
        seen[k] += 1
counters = sorted({c for v in rows.values() for c in v})
print("kernel#launch".ljust(28), *[c.replace("SQ_", "")[:13].rjust(13) for c in counters])
for (k, i), v in sorted(rows.items(), key=lambda x: (x[0][1], x[0][0])):
    print(f"{k[:24]}#{i}".ljust(28), *[f"{v.get(c, float('nan')):13.4g}" for c in counters])
