#!/bin/bash
# A/B of environment knobs on the headline bench (one GPU call): every argument is one configuration, a
# space-separated list of VAR=value settings ("" = the defaults); each runs bench.py under its own time limit and
# appends {"knobs": ..., "ms_per_step": ..., kernels} to gpurun_out/ab_<tag>.jsonl.
# usage: tools/ab_knobs.sh <tag> "<config 1>" "<config 2>" ...   (BENCH_ARGS: extra bench.py arguments)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/ab_$TAG.jsonl
mkdir -p "$R/gpurun_out"
: > "$OUT"
for cfg in "$@"; do
  env $cfg timeout -k 10 240 python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS \
    > "$R/gpurun_out/ab_$TAG.last.json" 2> "$R/gpurun_out/ab_$TAG.last.err"
  python3 - "$cfg" "$R/gpurun_out/ab_$TAG.last.json" >> "$OUT" <<'EOF'
import json, sys
line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(json.dumps({"knobs": sys.argv[1], "ms_per_step": line["ms_per_step"],
                  "check": (line.get("check") or {}).get("status"),
                  "kernels": {k: round(v["ms_per_launch"], 4) for k, v in line.get("kernels", {}).items()}}))
EOF
  tail -1 "$OUT"
done
