#!/bin/bash
# round-3 GPU check Y: TableScan workgroup size for 1-byte columns (HY_SCAN_SEG8 A/B), scan tests at each size
mkdir -p gpurun_out
for g in 2 4 8; do
  HY_SCAN_SEG8=$g timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3y_tests_$g.log 2>&1 || exit 1
  HY_SCAN_SEG8=$g timeout -k 10 200 python -u bench.py --workload scan --no-cpu-baseline --steps 20 > gpurun_out/r3y_scan_$g.json 2> gpurun_out/r3y_scan_$g.err || exit 2
done
