"""One-line summary of a bench.py JSON output: ms/step and per-kernel ms per launch. usage: bench_line.py TAG FILE"""
import json
import sys

d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = sorted(d["kernels"].items(), key=lambda kv: -kv[1]["ms_total"])
print(sys.argv[1], d["ms_per_step"], " ".join(f"{k}={v['ms_per_launch']:.3f}" for k, v in ks))
