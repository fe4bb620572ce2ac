#!/bin/bash
# Round profiles on the GPU box (run through gpurun from the repo root): per workload one rocprofv3 --kernel-trace
# --stats pass over the bench command, then separate FETCH_SIZE and WRITE_SIZE PMC passes (one counter each,
# restricted to the framework's kernels), summarised by tools/summarize_rocprof.py. A bench run executes warmup + K
# timed + K kernel-stats steps, so the PMC runs (--steps 2 --warmup 1) cover 5 steps. Every pass runs with
# HY_JOIN_OVERLAP=0 (the two join sides on one stream), so a partition kernel's traced duration is its own and not
# stretched by the other side's kernels running beside it. Each pass has its own time limit.
# usage: tools/profile_round.sh <tag> [workloads...]   (workloads: sf100 q1 q3 scan joinonly widen; default sf100 q1)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
shift || true
WL=${*:-sf100 q1}
export TMPDIR=/tmp
export HY_JOIN_OVERLAP=0
cd /tmp
run() {  # name, bench args
  local name=$1
  shift
  local OUT=$R/gpurun_out/prof_${TAG}_$name
  mkdir -p "$OUT"
  timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- \
    python3 "$R/bench.py" "$@" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_under_trace.json" 2> "$OUT/trace.err"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex 'hyk::|agg_jit' -d "$OUT/$c" -o run -f csv -- \
      python3 "$R/bench.py" "$@" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_under_$c.json" 2> "$OUT/$c.err"
  done
  python3 "$R/tools/summarize_rocprof.py" "$OUT" 5 > "$R/gpurun_out/${TAG}_rocprof_${name}_summary.json"
  cp "$OUT"/trace/run_kernel_stats.csv "$R/gpurun_out/${TAG}_rocprof_${name}_kernel_stats.csv"
  echo "profiled $name"
}
for w in $WL; do
  case $w in
    sf100) run sf100_fused ;;
    q1) run q1_sf100 --workload q1 ;;
    q3) run q3_sf100 --workload q3 ;;
    scan) run scan_sf10 --workload scan ;;
    joinonly) run joinonly_sf10 --workload join-only ;;
    widen)
      OUT=$R/gpurun_out/prof_${TAG}_widen
      mkdir -p "$OUT"
      timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- \
        python3 "$R/tools/bench_widen.py" --steps 3 > "$R/gpurun_out/${TAG}_widen_ops.jsonl" 2> "$OUT/trace.err"
      cp "$OUT"/trace/run_kernel_stats.csv "$R/gpurun_out/${TAG}_rocprof_widen_kernel_stats.csv"
      echo "profiled widen" ;;
  esac
done
