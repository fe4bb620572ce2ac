#!/bin/bash
# round-3 GPU check Z: 1-byte scans at 4 tiles per workgroup by default - GPU tests, scan / operator / TPC-H 3 benches
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --workload scan --no-cpu-baseline --steps 20 > gpurun_out/r3z_scan.json 2> gpurun_out/r3z_scan.err || exit 2
timeout -k 10 300 python -u bench.py --through-operators --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3z_ops.json 2> gpurun_out/r3z_ops.err || exit 3
timeout -k 10 300 python -u bench.py --workload q3 --no-cpu-baseline > gpurun_out/r3z_q3.json 2> gpurun_out/r3z_q3.err || exit 4
