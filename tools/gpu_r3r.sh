#!/bin/bash
# round-3 GPU check R: bench lines with the dominant-kernel roofline (timing pass without side-stream overlap)
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3r_bench.json 2> gpurun_out/r3r_bench.err || exit 1
timeout -k 10 300 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3r_q1.json 2> gpurun_out/r3r_q1.err || exit 2
