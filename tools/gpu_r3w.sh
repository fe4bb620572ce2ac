#!/bin/bash
# round-3 GPU check W: output chunks built while the join runs - GPU tests, then the operator path with phase traces
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3w_ops.json 2> gpurun_out/r3w_ops.err || exit 2
HY_OP_TRACE=1 timeout -k 10 400 python -u bench.py --through-operators --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r3w_ops_trace.json 2> gpurun_out/r3w_ops_trace.err || exit 3
