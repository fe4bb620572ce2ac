#!/bin/bash
# round-3 GPU check I: agg_dense_vec (aggregate tests, TPC-H 1 fused-scan bench at both register budgets, PMC)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_aggregate_lanes_gpu.py tests/test_aggregate_expr_gpu.py tests/test_aggregate_gpu.py tests/test_tpch_queries.py tests/test_scan_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3i_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3i_q1_fused.json 2> gpurun_out/r3i_q1_fused.err || exit 3
HY_VEC_OCC=4 timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3i_q1_fused_occ4.json 2> gpurun_out/r3i_q1_fused_occ4.err || exit 4
bash tools/pmc_lanes.sh q1vec --q1-fused > gpurun_out/r3i_pmc_vec.txt 2>&1 || exit 7
