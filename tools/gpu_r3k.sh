#!/bin/bash
# round-3 GPU check K: agg_dense_vec with per-period exactness: aggregate tests, TPC-H 1 fused-scan + PosList plans, PMC
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_aggregate_lanes_gpu.py tests/test_aggregate_expr_gpu.py tests/test_aggregate_gpu.py tests/test_tpch_queries.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3k_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3k_q1_fused.json 2> gpurun_out/r3k_q1_fused.err || exit 3
bash tools/pmc_lanes.sh q1vec5 --q1-fused > gpurun_out/r3k_pmc_vec.txt 2>&1 || exit 7
