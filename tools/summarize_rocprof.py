"""Condenses a tools/profile_bench.sh output directory into one JSON summary per kernel:

- from the --kernel-trace --stats pass: calls and average duration (ns) per kernel,
- from the FETCH_SIZE / WRITE_SIZE passes: HBM bytes per launch. rocprofv3 reports both in KiB
  (derived_counters.xml: TCC_EA0_RDREQ/_WRREQ requests x 32/64 B / 1024). Following
  /opt/skills/guides/MI355X_MICROARCH.md (HBM section), FETCH_SIZE on gfx950 tallies 128-B requests at 64 B, so
  the read bytes are doubled; WRITE_SIZE is taken as is.

Kernel names are shortened to the framework's kernel function name (hyk::<name>) so they line up with bench.py's
per-kernel table; a partition kernel's side comes from its template tag (hyk::OnBuild / hyk::OnProbe), so each launch
is attributed from its own name.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    """hyk::<kernel>, plus .build / .probe / .exchange for the partition kernels, whose first template argument
    (hyk::OnBuild / hyk::OnProbe / hyk::OnExchange) names the join side of the launch."""
    m = re.search(r"hyk::(\w+)", name)
    if not m:
        return name[:60]
    side = re.search(r"hyk::On(Build|Probe|Exchange)", name)
    return m.group(1) + ("." + side.group(1).lower() if side else "")


def one(pattern):
    files = sorted(glob.glob(pattern, recursive=True))
    return files[-1] if files else None


def main(out, steps=None):
    res = {"kernels": {}}
    stats = one(os.path.join(out, "trace", "**", "*kernel_stats.csv"))
    if stats:
        acc = defaultdict(lambda: [0, 0.0])
        with open(stats) as f:
            for row in csv.DictReader(f):
                k = short(row["Name"])
                acc[k][0] += int(row["Calls"])
                acc[k][1] += float(row["TotalDurationNs"])
        for k, (calls, tot) in acc.items():
            res["kernels"].setdefault(k, {}).update(calls=calls, avg_ns=tot / calls, total_ns=tot)
    for counter, scale in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        f = one(os.path.join(out, counter, "**", "*counter_collection.csv"))
        if not f:
            continue
        per_dispatch = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                d = row["Dispatch_Id"]
                per_dispatch[d] += float(row["Counter_Value"])
                names[d] = short(row["Kernel_Name"])
        by_kernel = defaultdict(list)
        for d, v in per_dispatch.items():
            by_kernel[names[d]].append(v * 1024.0 * scale)
        key = "hbm_read_bytes_per_launch" if counter == "FETCH_SIZE" else "hbm_write_bytes_per_launch"
        for k, vals in by_kernel.items():
            res["kernels"].setdefault(k, {})[key] = sum(vals) / len(vals)
            res["kernels"][k][key.replace("per_launch", "launches")] = len(vals)
    for k, v in res["kernels"].items():
        if "hbm_read_bytes_per_launch" in v and "hbm_write_bytes_per_launch" in v:
            v["hbm_bytes_per_launch"] = v["hbm_read_bytes_per_launch"] + v["hbm_write_bytes_per_launch"]
    if steps:  # the PMC runs' steps (warmup + timed): HBM bytes of one step over every kernel of the path
        total = 0.0
        for k, v in res["kernels"].items():
            if k.startswith("stream_") or "hbm_bytes_per_launch" not in v:
                continue  # the roofline probe is not part of a step
            total += v["hbm_bytes_per_launch"] * v.get("hbm_read_bytes_launches", 0)
        res["hbm_bytes_per_step"] = total / steps
        res["pmc_steps"] = steps
    res["corrections"] = "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), WRITE_SIZE x1; KiB -> bytes"
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
