"""Instruction mix of one kernel in a hipcc -S device assembly file: python tools/asm_mix.py FILE.s SYMBOL_SUBSTRING."""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
names = [l.split(":")[0] for l in lines if re.match(r"^[A-Za-z_]\S*:", l) and sys.argv[2] in l.split(":")[0]]
for name in names:
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cnt = collections.Counter()
    for l in lines[start:end]:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_")
               else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
        cnt[cls] += 1
        cnt[op] += 1
    meta = {k: re.search(r", (\d+)", l).group(1) for l in lines for k in ("num_vgpr", "private_seg_size")
            if l.startswith("\t.set " + name + "." + k)}
    print(name[:90], {k: cnt[k] for k in ("valu", "salu", "lds", "vmem")}, meta)
    if len(sys.argv) > 3:
        for k, v in cnt.most_common(int(sys.argv[3])):
            print("   ", k, v)
