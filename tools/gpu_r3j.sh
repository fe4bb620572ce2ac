#!/bin/bash
# round-3 GPU check J: wave-uniform wave index in every kernel + agg_dense_vec: aggregate / scan / join tests, TPC-H 1
# fused-scan bench at both register budgets, headline bench, PMC of agg_dense_vec
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_aggregate_lanes_gpu.py tests/test_aggregate_expr_gpu.py tests/test_aggregate_gpu.py tests/test_tpch_queries.py tests/test_scan_gpu.py tests/test_join_gpu.py tests/test_scan_join_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3j_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) exit 1;; esac
timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3j_q1_fused.json 2> gpurun_out/r3j_q1_fused.err || exit 3
HY_VEC_OCC=4 timeout -k 10 240 python -u bench.py --workload q1 --q1-fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3j_q1_fused_occ4.json 2> gpurun_out/r3j_q1_fused_occ4.err || exit 4
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || exit 5
bash tools/pmc_lanes.sh q1vec --q1-fused > gpurun_out/r3j_pmc_vec.txt 2>&1 || exit 7
