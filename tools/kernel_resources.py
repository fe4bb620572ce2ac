"""Summarize hipcc -Rpass-analysis=kernel-resource-usage for the C-ABI library (one line per kernel)."""
import re
import subprocess
import sys

cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude", "-c",
       "TU", "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"]
out = ""
for tu in ("hyrise-1_amd/csrc/capi/hyrise_amd.hip", "hyrise-1_amd/csrc/capi/hyrise_amd_aggregate.hip",
           "hyrise-1_amd/csrc/capi/hyrise_amd_join_i32.hip"):
    if len(sys.argv) > 2 and sys.argv[2] not in tu:
        continue
    out += subprocess.run([tu if a == "TU" else a for a in cmd], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "SGPRs", "ScratchSize \[bytes/lane\]", "Occupancy \[waves/SIMD\]", "LDS Size \[bytes/block\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
filt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if filt in r["name"]:
        print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs')} sgpr={r.get('SGPRs')} scratch={r.get('ScratchSize')} "
              f"occ={r.get('Occupancy')} lds={r.get('LDS')}")
