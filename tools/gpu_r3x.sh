#!/bin/bash
# round-3 GPU check X: operator path phase traces (output builders' own time), thread-count A/B
mkdir -p gpurun_out
for t in 16 8; do
  HY_OP_THREADS=$t HY_OP_TRACE=1 timeout -k 10 300 python -u bench.py --through-operators --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r3x_ops_t$t.json 2> gpurun_out/r3x_ops_t$t.err || exit 1
done
