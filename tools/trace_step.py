"""Timeline of one bench step from a rocprofv3 kernel trace: every kernel between the last two `join_partition`
launches (or the last N kernels), with its duration, the idle gap before it, VGPRs and grid; then per-name totals.
usage: python tools/trace_step.py <run_kernel_trace.csv> [anchor-regex] [--all]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"hyk::(\w+)(<[^(]*>)?", name)
    if not m:
        return name[:60]
    base = m.group(1)
    args = m.group(2) or ""
    tag = "build" if "OnBuild" in args else "probe" if "OnProbe" in args else "exch" if "OnExchange" in args else ""
    return base + ("." + tag if tag else "")


def main():
    path = sys.argv[1]
    anchor = re.compile(sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else r"join_partition<")
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor.search(r["Kernel_Name"])]
    if len(idx) < 2:
        print("anchor not found twice")
        return
    lo, hi = idx[-2] + 1, idx[-1] + 1
    # include the trailing list kernels after the anchor (multi / skewed) up to the next non-join kernel
    while hi < len(rows) and "join_partition" in rows[hi]["Kernel_Name"]:
        hi += 1
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = int(rows[lo - 1]["End_Timestamp"])
    tot = defaultdict(lambda: [0, 0.0])
    show = "--all" in sys.argv
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = short(r["Kernel_Name"])
        tot[n][0] += 1
        tot[n][1] += (e - s) / 1e3
        if show or (e - s) > 5000:
            print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:6.1f}  "
                  f"vgpr {r['VGPR_Count']:>4} grid {int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])):>7}  {n}")
        prev_end = max(prev_end, e)
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
    busy = sum(v[1] for v in tot.values())
    print(f"step span {span:.1f} us, kernel busy {busy:.1f} us, launches {len(step)}")
    for n, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"  {n:40s} {c:4d} launches {us:9.1f} us")


if __name__ == "__main__":
    main()
