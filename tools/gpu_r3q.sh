#!/bin/bash
# round-3 GPU check Q: operator path output-chunk construction A/B: builder threads x glibc trimming
mkdir -p gpurun_out
for cfg in "1 0" "16 0" "1 1" "16 1"; do
  set -- $cfg
  if [ "$2" = 1 ]; then export MALLOC_TRIM_THRESHOLD_=100000000000 MALLOC_TOP_PAD_=1000000000 MALLOC_MMAP_THRESHOLD_=100000000000; else unset MALLOC_TRIM_THRESHOLD_ MALLOC_TOP_PAD_ MALLOC_MMAP_THRESHOLD_; fi
  HY_OP_THREADS=$1 HY_OP_TRACE=1 timeout -k 10 300 python -u bench.py --through-operators --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r3q_ops_t$1_m$2.json 2> gpurun_out/r3q_ops_t$1_m$2.err || exit 2
done
