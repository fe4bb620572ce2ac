#!/bin/bash
# round-3 GPU check G: fixed string / compressed-scan tests, filtered-pass A/B (match bits with 1-tile spans), TPC-H 1
# variants (default / RowID prefetch / fused scan)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py tests/test_string_scan_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3g_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
HY_PART_SUB_FILTERED=1 timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3g_bench_mask_sub1.json 2> gpurun_out/r3g_bench_mask_sub1.err || exit 2
timeout -k 10 240 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3g_q1.json 2> gpurun_out/r3g_q1.err || exit 3
HY_AGG_PREFETCH=1 timeout -k 10 240 python -u bench.py --workload q1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3g_q1_pf.json 2> gpurun_out/r3g_q1_pf.err || exit 4
timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3g_q1_fused.json 2> gpurun_out/r3g_q1_fused.err || exit 5
bash tools/pmc_lanes.sh q1 > gpurun_out/r3g_pmc_lanes.txt 2>&1 || exit 6
bash tools/pmc_lanes.sh q1fused --q1-fused > gpurun_out/r3g_pmc_lanes_fused.txt 2>&1 || exit 7
