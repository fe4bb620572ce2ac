#!/bin/bash
# Profiles the default bench.py run on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats over the exact default bench command (per-kernel average durations, to be
#      compared with bench.py's live HIP-event timings),
#   2. two separate PMC passes, FETCH_SIZE and WRITE_SIZE (they do not fit one pass on gfx950), restricted to the
#      framework's kernels,
# then writes <out>/summary.json via tools/summarize_rocprof.py.
# usage: tools/profile_bench.sh <out-dir under gpurun_out> [bench args for the PMC passes]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/prof}
shift || true
PMC_ARGS=${*:-"--steps 2 --warmup 1 --no-cpu-baseline"}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- \
  python3 "$R/bench.py" > "$OUT/bench_under_trace.json" 2> "$OUT/trace.err"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 420 rocprofv3 --pmc $c --kernel-include-regex 'hyk::' -d "$OUT/$c" -o run -f csv -- \
    python3 "$R/bench.py" $PMC_ARGS > "$OUT/bench_under_$c.json" 2> "$OUT/$c.err"
done
python3 "$R/tools/summarize_rocprof.py" "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
