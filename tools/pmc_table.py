"""Per-kernel table of rocprofv3 --pmc counters (summed over dimensions, averaged over dispatches of the same
kernel name). usage: pmc_table.py <run_counter_collection.csv> [...]"""
import collections
import csv
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        vals[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add((path, r["Dispatch_Id"]))
counters = sorted({c for v in vals.values() for c in v})
print("kernel".ljust(40), "n", *[c.replace("SQ_", "")[:14].rjust(14) for c in counters])
for k, v in sorted(vals.items()):
    n = len(disp[k]) / len(sys.argv[1:])
    print(k.ljust(40), int(n), *[f"{v[c] / n:14.4g}" for c in counters])
