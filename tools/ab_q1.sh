#!/bin/bash
# A/B of environment settings on the TPC-H 1 bench (one GPU call): every argument is one configuration ("" = the
# defaults); each runs `bench.py --workload q1` under its own time limit and appends {"knobs", "ms_per_step", kernels}
# to gpurun_out/ab_q1_<tag>.jsonl. usage: tools/ab_q1.sh <tag> "<config 1>" "<config 2>" ...
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/ab_q1_$TAG.jsonl
mkdir -p "$R/gpurun_out"
: > "$OUT"
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python3 "$R/bench.py" --workload q1 --steps 10 --warmup 3 --no-cpu-baseline \
    > "$R/gpurun_out/ab_q1_$TAG.last.json" 2> "$R/gpurun_out/ab_q1_$TAG.last.err"
  python3 - "$cfg" "$R/gpurun_out/ab_q1_$TAG.last.json" >> "$OUT" <<'PY'
import json, sys
line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(json.dumps({"knobs": sys.argv[1], "ms_per_step": line["ms_per_step"], "check": (line.get("check") or {}).get("ok"),
                  "kernels": {k: round(v["ms_per_launch"], 4) for k, v in line.get("kernels", {}).items()}}))
PY
  tail -1 "$OUT"
done
